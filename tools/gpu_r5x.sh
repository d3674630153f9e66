#!/bin/bash
# Round 5, call x: validator-mode step pipelines (--vpipes 1 / 2 / 3) after the
# state-machine rework, alternating, one rank.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 HBRBC_JIT=load
OUT=gpurun_out/r5x
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
for rep in 1 2; do
  for P in 2 1 3; do
    timeout -k 10 300 python bench.py --mode validators --vpipes $P --steps 10 --warmup 3 --no-cpu --no-riders --f4-checks 0 > $OUT/b_${P}_${rep}.log 2>&1
    rc=$?; if fatal $rc; then exit $rc; fi
    grep '^{' $OUT/b_${P}_${rep}.log | tail -1 | python3 -c "
import json,sys; d=json.load(sys.stdin)
print('vpipes $P', round(d['validators']['value'],2), round(d['validators']['ms_per_step'],3), 'cfg4', round(d['validators_cfg4']['value'],2), round(d['validators_cfg4']['ms_per_step'],3))" | tee -a $OUT/summary.txt
  done
done
exit 0
