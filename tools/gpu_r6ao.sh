#!/bin/bash
# Round 6, call ao: the pairing tests with the G2 preparation's cross-block case.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out/r6ao
timeout -k 10 400 python -u -m pytest tests/test_pairing.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r6ao/tests.log 2>&1
rc=$?; echo "tests exit $rc"; grep -E "PASS|FAIL|ERROR|passed|failed|assert" gpurun_out/r6ao/tests.log | tail -30
exit $rc
