#!/bin/bash
# Round 4, call aa: validator-mode proposals per step (cfg3 4096 vs 8192,
# cfg4 2048 vs 4096) with the default schedule (overlap, two step pipelines).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp HBRBC_JIT=load
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
for i in 1 2; do
  for V in cfg3:4096 cfg3:8192 cfg4:2048 cfg4:4096; do
    C=${V%%:*}; N=${V#*:}
    timeout -k 10 300 python bench.py --mode validators --config $C --vcount $N --steps 10 --warmup 2 --no-cpu --f4-checks 0 > gpurun_out/r4aa_${C}_${N}_$i.log 2>&1
    rc=$?; echo "$C vcount $N run $i exit $rc"; if fatal $rc; then exit $rc; fi
    grep '^{' gpurun_out/r4aa_${C}_${N}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['validators']; print('   ', round(d['value'], 2), round(d['ms_per_step'], 3))"
  done
done
exit 0
