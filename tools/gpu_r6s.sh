#!/bin/bash
# Round 6, call s: f4 leg with the key preparation on a side stream (beside the
# G2 preparation) vs serial, alternating, small headline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 HBRBC_JIT=load
OUT=gpurun_out/r6s
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
for rep in 1 2 3; do
for S in 0 1; do
  HBRBC_BENCH_F4_SIDE=$S timeout -k 10 300 python bench.py --mode instances --no-riders --no-leaf-reuse --no-cpu --count 1024 --steps 2 --f4-steps 6 > $OUT/f4_s${S}_${rep}.log 2>&1
  rc=$?; if fatal $rc; then exit $rc; fi
  grep '^{' $OUT/f4_s${S}_${rep}.log | tail -1 | python3 -c "
import json,sys; d=json.load(sys.stdin); t=d['threshold_decrypt']
print('side=$S rep=$rep', t.get('value'), t.get('ms_per_step'), t.get('error'))" | tee -a $OUT/summary.txt
done
done
exit 0
