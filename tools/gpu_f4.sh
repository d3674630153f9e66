#!/bin/bash
# f4 (pairing) GPU parity tests, then the full GPU suite and the bench round trip.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_pairing.py -x -v --timeout 240 --timeout-method thread > gpurun_out/f4_tests.log 2>&1
rc=$?; echo "f4 tests exit $rc"; tail -15 gpurun_out/f4_tests.log
exit $rc
