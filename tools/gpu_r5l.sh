#!/bin/bash
# Round 5, call l: state-machine launch forms re-measured with the round-5
# inbox cursor and predicated Echo handler (sm_bench, alternating).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/r5l
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
for rep in 1 2; do
  for V in "X=0" "HBRBC_SM_W4=0" "HBRBC_SM_GREC=0" "HBRBC_SM_GREC=1" "HBRBC_SM_STAGED=0"; do
    env $V timeout -k 10 120 python tools/sm_bench.py --reps 7 2>/dev/null | sed "s/^/$V /" >> $OUT/sm_forms.txt
    rc=$?; if fatal $rc; then exit $rc; fi
  done
done
cat $OUT/sm_forms.txt | python3 -c "
import sys, json
for l in sys.stdin:
    v, j = l.split(' ', 1); d = json.loads(j); print('%-20s n=%3d %.3f ms' % (v, d['n'], d['ms_median']))"
exit 0
