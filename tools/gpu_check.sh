#!/bin/bash
# GPU round-trip used during development: parity tests, smoke, short bench.
# Stops at the first step that faults, aborts or times out.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests exit $rc"; tail -3 gpurun_out/gpu_tests.log
if fatal $rc; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke exit $rc"; tail -2 gpurun_out/smoke.log
if fatal $rc; then exit $rc; fi
timeout -k 10 300 python bench.py ${BENCH_ARGS:---steps 5 --warmup 1 --cpu-seconds 5} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench exit $rc"; tail -c 3000 gpurun_out/bench.log
exit $rc
