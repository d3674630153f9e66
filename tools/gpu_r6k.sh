#!/bin/bash
# Round 6, call k: cfg5 batch / pipelines A/B (2048 vs 4096 instances, 2048 x 2 pipelines).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 HBRBC_JIT=load
OUT=gpurun_out/r6k
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
for rep in 1 2; do
for V in "c2048:--count 2048" "c4096:--count 4096" "p2:--count 2048 --ipipes 2"; do
  n=${V%%:*}; a=${V#*:}
  timeout -k 10 300 python bench.py --config cfg5 --mode instances --no-cpu --f4-checks 0 $a > $OUT/cfg5_${n}_${rep}.log 2>&1
  rc=$?; if fatal $rc; then exit $rc; fi
  grep '^{' $OUT/cfg5_${n}_${rep}.log | tail -1 | python3 -c "
import json,sys; d=json.load(sys.stdin)
print('cfg5 $n rep=$rep', d['value'], d['ms_per_step'], d['roofline']['frac'], {k: round(v,2) for k,v in d['stages_ms_per_step'].items()})" | tee -a $OUT/summary.txt
done
done
exit 0
