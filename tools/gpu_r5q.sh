#!/bin/bash
# Round 5, call q: inbox prefetch in the state machine's sender loop
# (HB_SM_PREFETCH=1 default; hbbft_amd/ab/libhbrbc_nopf.so built with 0) on
# top of the lean kernels -- parity of every form, then sm_bench alternating
# the two libraries and the lean switch.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
export PYTHONUNBUFFERED=1 TMPDIR=/tmp HBRBC_JIT_DIR=$ROOT/hbbft_amd/jit
OUT=gpurun_out/r5q
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 700 python -u -m pytest tests/test_rbc_sim.py tests/test_sharded.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests exit $rc"; tail -3 $OUT/tests.log; if fatal $rc; then exit $rc; fi
[ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do
  for V in "libhbrbc.so 1" "ab/libhbrbc_nopf.so 1" "libhbrbc.so 0"; do
    set -- $V
    HBRBC_LIB=$ROOT/hbbft_amd/$1 HBRBC_SM_LEAN=$2 timeout -k 10 120 python tools/sm_bench.py --reps 7 > $OUT/b.json 2>/dev/null
    rc=$?; if fatal $rc; then exit $rc; fi
    sed "s/^{/{\"lean\": $2, /" $OUT/b.json >> $OUT/sm_bench.jsonl
  done
done
cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace -d $ROOT/$OUT/trace -o run -- python3 $ROOT/tools/sm_bench.py --reps 2 > $ROOT/$OUT/trace.log 2>&1
rc=$?; cd $ROOT; echo "trace exit $rc"; if fatal $rc; then exit $rc; fi
python3 -c "
import json
for l in open('$OUT/sm_bench.jsonl'):
    d = json.loads(l); print(d['lib'], 'lean', d['lean'], d['n'], round(d['ms_median'], 3), round(d['ms_min'], 3))
"
exit 0
