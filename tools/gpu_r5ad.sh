#!/bin/bash
# Round 5, call ad: validator objects with the data-plane streams at high
# priority (HBRBC_BENCH_MAIN_PRIO=1) vs default priorities, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 HBRBC_JIT=load
OUT=gpurun_out/r5ad
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
python3 -c "import torch; print('priority range', torch.cuda.Stream.priority_range())"
for rep in 1 2; do
  for P in 0 1; do
    HBRBC_BENCH_MAIN_PRIO=$P timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu --no-riders --f4-checks 0 > $OUT/b_${P}_${rep}.log 2>&1
    rc=$?; if fatal $rc; then exit $rc; fi
    grep '^{' $OUT/b_${P}_${rep}.log | tail -1 | python3 -c "
import json,sys; d=json.load(sys.stdin)
print('prio $P', 'head', round(d['value'],2), 'validators', round(d['validators']['value'],2), 'cfg4', round(d['validators_cfg4']['value'],2))" | tee -a $OUT/summary.txt
  done
done
exit 0
