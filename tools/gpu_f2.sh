#!/bin/bash
# f2 state-machine tests on the GPU, then the usual round trip (tools/gpu_round.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 600 python -u -m pytest tests/test_rbc_sim.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/${TAG:-r3}_sm_tests.log 2>&1
rc=$?; echo "sm tests exit $rc"; tail -30 gpurun_out/${TAG:-r3}_sm_tests.log
if fatal $rc; then exit $rc; fi
PYTEST_ARGS="--ignore=tests/test_rbc_sim.py" bash tools/gpu_round.sh
