#!/bin/bash
# Round 4, call ah: --vpipes 1 vs 2 at the final validator batches (cfg3 8192,
# cfg4 4096 proposals per step).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp HBRBC_JIT=load
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
for i in 1 2; do
  for C in cfg3 cfg4; do
    for P in 1 2; do
      timeout -k 10 300 python bench.py --mode validators --config $C --steps 10 --warmup 2 --no-cpu --f4-checks 0 --vpipes $P > gpurun_out/r4ah_${C}_p${P}_$i.log 2>&1
      rc=$?; echo "$C vpipes $P run $i exit $rc"; if fatal $rc; then exit $rc; fi
      grep '^{' gpurun_out/r4ah_${C}_p${P}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['validators']; print('   ', round(d['value'], 2), round(d['ms_per_step'], 3))"
    done
  done
done
exit 0
