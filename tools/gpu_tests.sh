#!/bin/bash
# GPU parity tests only (fast round trip during development); stops at the
# first fatal status.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests exit $rc"; tail -15 gpurun_out/gpu_tests.log
exit $rc
