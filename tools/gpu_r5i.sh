#!/bin/bash
# Round 5, call i: the select-form Echo handler (HB_SM_SELECT=1,
# hbbft_amd/ab/libhbrbc_sel.so) -- parity of every state-machine form
# against the host restatement, then sm_bench alternating with the default.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
export PYTHONUNBUFFERED=1 TMPDIR=/tmp HBRBC_JIT_DIR=$ROOT/hbbft_amd/jit
OUT=gpurun_out/r5i
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
HBRBC_LIB=$ROOT/hbbft_amd/ab/libhbrbc_sel.so timeout -k 10 600 python -u -m pytest tests/test_rbc_sim.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests_sel.log 2>&1
rc=$?; echo "tests (select form) exit $rc"; tail -2 $OUT/tests_sel.log; if fatal $rc; then exit $rc; fi
[ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do
  for L in libhbrbc.so ab/libhbrbc_sel.so; do
    HBRBC_LIB=$ROOT/hbbft_amd/$L timeout -k 10 120 python tools/sm_bench.py --reps 7 >> $OUT/sm_bench.jsonl 2>/dev/null
    rc=$?; if fatal $rc; then exit $rc; fi
  done
done
python3 -c "
import json
for l in open('$OUT/sm_bench.jsonl'):
    d = json.loads(l); print(d['lib'], d['n'], round(d['ms_median'], 3))
"
exit 0
