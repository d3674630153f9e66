#!/bin/bash
# Round 3z: every GPU test with the cfg4 pass shapes (two encoder programs of
# 6-row passes, 7-row generic reconstruct), cfg4 bench line, default line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3z_tests.log 2>&1
rc=$?; echo "tests exit $rc"; tail -2 gpurun_out/r3z_tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3z_smoke.log 2>&1
rc=$?; echo "smoke exit $rc"; if [ $rc -ne 0 ]; then exit $rc; fi
export HBRBC_JIT=load
timeout -k 10 400 python bench.py --config cfg4 --steps 5 --warmup 1 --f4-checks 0 --mode instances --cpu-seconds 2 --cpu-reps 3 > gpurun_out/r3z_bench_cfg4.log 2>&1
rc=$?; echo "bench cfg4 exit $rc"; if fatal $rc; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/r3z_bench.log 2>&1
rc=$?; echo "bench exit $rc"
exit $rc
