#!/bin/bash
# Round 5, call w: the generic reconstruct's set-bit layout (HBRBC_GF=
# bitslice_likely: __builtin_expect(bit, 1), the set-bit XORs inline) against
# the default (out-of-line bodies), alternating, instance mode cfg3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 HBRBC_JIT=load
OUT=gpurun_out/r5w
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
for rep in 1 2; do
  for M in default bitslice_likely; do
    if [ $M = default ]; then unset HBRBC_GF; else export HBRBC_GF=$M; fi
    timeout -k 10 300 python bench.py --mode instances --steps 6 --warmup 2 --no-cpu --no-riders --f4-checks 0 > $OUT/b_${M}_${rep}.log 2>&1
    rc=$?; if fatal $rc; then exit $rc; fi
    grep '^{' $OUT/b_${M}_${rep}.log | tail -1 | python3 -c "
import json,sys; d=json.load(sys.stdin); s=d['stages_ms_per_step']
print('$M', round(d['value'],2), 'reconstruct', round(s['reconstruct'],3), 'encode', round(s['encode'],3))" | tee -a $OUT/summary.txt
  done
done
exit 0
