#!/bin/bash
# Round 6, call f: step pipelines on the contexts' own streams for the cfg3
# headline (--ipipes 1 / 2) and the validator objects (HBRBC_BENCH_OWNQ 0 / 1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 HBRBC_JIT=load
OUT=gpurun_out/r6f
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
for rep in 1 2; do
for P in 1 2; do
  timeout -k 10 300 python bench.py --mode instances --ipipes $P --no-leaf-reuse --no-cpu --f4-checks 0 > $OUT/cfg3_p${P}_${rep}.log 2>&1
  rc=$?; if fatal $rc; then exit $rc; fi
  grep '^{' $OUT/cfg3_p${P}_${rep}.log | tail -1 | python3 -c "
import json,sys; d=json.load(sys.stdin)
print('cfg3 pipes=$P rep=$rep', d['value'], d['ms_per_step'], {k: round(v,2) for k,v in d['stages_ms_per_step'].items()})" | tee -a $OUT/summary.txt
done
for Q in 0 1; do
  HBRBC_BENCH_OWNQ=$Q timeout -k 10 300 python bench.py --mode validators --no-cpu --f4-checks 0 > $OUT/val_q${Q}_${rep}.log 2>&1
  rc=$?; if fatal $rc; then exit $rc; fi
  HBRBC_BENCH_OWNQ=$Q timeout -k 10 300 python bench.py --mode validators --config cfg4 --no-cpu --f4-checks 0 > $OUT/val4_q${Q}_${rep}.log 2>&1
  rc=$?; if fatal $rc; then exit $rc; fi
  for f in val val4; do grep '^{' $OUT/${f}_q${Q}_${rep}.log | tail -1 | python3 -c "
import json,sys; d=json.load(sys.stdin)
print('$f ownq=$Q rep=$rep', d['value'], d['ms_per_step'])" | tee -a $OUT/summary.txt; done
done
done
# the 4-rank gloo rehearsal of the multi-GPU line on the new phase order
HBRBC_BENCH_REHEARSE=1 timeout -k 10 900 python bench.py --gpus 4 --steps 2 --warmup 1 --f4-checks 65536 --phase-budget 800 --detail $OUT/detail_g4.json > $OUT/rehearsal_g4.log 2>&1
rc=$?; echo "rehearsal g4 exit $rc"; grep '^{' $OUT/rehearsal_g4.log | tail -1 > $OUT/rehearsal_g4.json; wc -c $OUT/rehearsal_g4.json
exit $rc
