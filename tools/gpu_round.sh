#!/bin/bash
# One GPU round trip: parity tests, smoke, the default bench line, and a
# 2-rank gloo rehearsal of the multi-GPU line with hiprtc compiles forbidden
# (HBRBC_JIT=load: every code object the bench needs must come from build()).
# Stops at the first step that faults, aborts or times out.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
TAG=${TAG:-r3}
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/${TAG}_gpu_tests.log 2>&1
  rc=$?; echo "tests exit $rc"; tail -3 gpurun_out/${TAG}_gpu_tests.log
  if fatal $rc; then exit $rc; fi
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
  rc=$?; echo "smoke exit $rc"; tail -2 gpurun_out/${TAG}_smoke.log
  if fatal $rc; then exit $rc; fi
fi
HBRBC_JIT=load timeout -k 10 600 python bench.py ${BENCH_ARGS:---steps 10 --warmup 2} > gpurun_out/${TAG}_bench.log 2>&1
rc=$?; echo "bench exit $rc"; tail -c 1500 gpurun_out/${TAG}_bench.log
if fatal $rc; then exit $rc; fi
if [ -z "$SKIP_REHEARSAL" ]; then
  HBRBC_JIT=load HBRBC_BENCH_REHEARSE=1 timeout -k 10 600 python bench.py --gpus 2 --steps 3 --warmup 1 --f4-checks 65536 > gpurun_out/${TAG}_rehearsal_g2.log 2>&1
  rc=$?; echo "rehearsal exit $rc"; tail -c 1500 gpurun_out/${TAG}_rehearsal_g2.log
fi
exit $rc
