#!/bin/bash
# Round 6, call af: the one-rank RCCL run of the bench's collective calls
# (tests/rccl_one_rank.py) and the sharded GPU tests around it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/r6af
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_sharded.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests exit $rc"; grep -E "PASS|FAIL|ERROR|passed|failed" $OUT/tests.log | tail -30
exit $rc
