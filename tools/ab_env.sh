#!/bin/bash
# A/B of environment knobs over bench configurations, one bench run each:
#   VAR=HBRBC_JIT_SYNC VALUES="0 2 4" CONFIGS="cfg5 cfg3" bash tools/ab_env.sh
#   SETS="HBRBC_RT_SPEC=14 HBRBC_RT_SPEC=11,HBRBC_JIT_FDEPTH=4" bash tools/ab_env.sh
# (SETS: each word one comma-separated list of VAR=value assignments)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
if [ -z "$SETS" ]; then
  SETS=""
  for v in ${VALUES}; do SETS="$SETS $VAR=$v"; done
fi
for c in ${CONFIGS:-cfg3}; do
  for s in ${SETS}; do
    tag=$(echo "$s" | tr ',=/.' '____')
    log=gpurun_out/ab/${c}_${tag}.log
    env $(echo "$s" | tr ',' ' ') timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-4} --warmup 1 --no-cpu --mode ${MODE:-instances} > $log 2>&1
    rc=$?
    python3 -c "
import json
l=[x for x in open('$log') if x.startswith('{')]
if not l: print('$c $s rc=$rc', open('$log').read()[-800:])
else:
  d=json.loads(l[-1]); st=d['stages_ms_per_step']
  print('$c $s  %.2f GB/s  %.2f ms/step  encode %.2f  reconstruct %.2f  leaf %.2f  validate %.2f' % (d['value'], d['ms_per_step'], st['encode'], st['reconstruct'], st['leaf_hash'], st['validate']))
"
    case $rc in 0) ;; *) exit $rc;; esac
  done
done
