#!/bin/bash
# A/B kernel variants on the default bench config: VARIANTS="ENV=.. --arg;ENV2=.." (';'-separated)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
IFS=';' read -ra VS <<< "${VARIANTS:-HBRBC_GF=bitslice;HBRBC_GF=perm}"
for v in "${VS[@]}"; do
  envs=$(echo $v | tr ' ' '\n' | grep = | tr '\n' ' ')
  args=$(echo $v | tr ' ' '\n' | grep -v = | tr '\n' ' ')
  echo "== $v"
  env $envs timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu $args > gpurun_out/bv.log 2>&1
  rc=$?
  python3 -c "
import json
l=[x for x in open('gpurun_out/bv.log') if x.startswith('{')]
d=json.loads(l[-1]); print(round(d['value'],2),'GB/s', round(d['ms_per_step'],2),'ms', {k:round(v,2) for k,v in d['stages_ms_per_step'].items()})
" || tail -5 gpurun_out/bv.log
  case $rc in 0) ;; *) echo "rc=$rc"; exit $rc;; esac
done
