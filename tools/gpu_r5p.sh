#!/bin/bash
# Round 5, call p: the lean state-machine kernels (rounds >= 2 of a batch
# without injected broadcasts run without the Value / Fake handlers) --
# parity of every form against the host restatement, then sm_bench
# alternating HBRBC_SM_LEAN=0 with the default.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
export PYTHONUNBUFFERED=1 TMPDIR=/tmp HBRBC_JIT_DIR=$ROOT/hbbft_amd/jit
OUT=gpurun_out/r5p
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 700 python -u -m pytest tests/test_rbc_sim.py tests/test_sharded.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests exit $rc"; tail -3 $OUT/tests.log; if fatal $rc; then exit $rc; fi
[ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do
  for L in 0 1; do
    HBRBC_SM_LEAN=$L timeout -k 10 120 python tools/sm_bench.py --reps 7 > $OUT/b.json 2>/dev/null
    rc=$?; if fatal $rc; then exit $rc; fi
    sed "s/^{/{\"lean\": $L, /" $OUT/b.json >> $OUT/sm_bench.jsonl
  done
done
python3 -c "
import json
for l in open('$OUT/sm_bench.jsonl'):
    d = json.loads(l); print('lean', d['lean'], d['n'], round(d['ms_median'], 3), round(d['ms_min'], 3))
"
exit 0
