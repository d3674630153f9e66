#!/bin/bash
# Round 5, call m: the state machine's w4 kernel forms at 5 and 6 waves/SIMD
# (hbbft_amd/ab/libhbrbc_w{5,6}.so, -DHB_SM_W4_WAVES) against the default 4.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
export PYTHONUNBUFFERED=1 TMPDIR=/tmp HBRBC_JIT_DIR=$ROOT/hbbft_amd/jit
OUT=gpurun_out/r5m
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
for rep in 1 2; do
  for L in libhbrbc.so ab/libhbrbc_w5.so ab/libhbrbc_w6.so; do
    HBRBC_LIB=$ROOT/hbbft_amd/$L timeout -k 10 120 python tools/sm_bench.py --reps 7 >> $OUT/sm.jsonl 2>/dev/null
    rc=$?; if fatal $rc; then exit $rc; fi
  done
done
python3 -c "
import json
for l in open('$OUT/sm.jsonl'):
    d = json.loads(l); print('%-18s n=%3d %.3f ms' % (d['lib'], d['n'], d['ms_median']))"
exit 0
