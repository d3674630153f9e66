#!/bin/bash
# Round 4, call ae: cfg3 instances per step beyond 32768 (49152, 65536).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp HBRBC_JIT=load
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
for i in 1 2; do
  for C in 32768 65536 49152; do
    timeout -k 10 400 python bench.py --mode instances --count $C --steps 6 --warmup 2 --no-cpu --f4-checks 0 --no-leaf-reuse > gpurun_out/r4ae_c${C}_$i.log 2>&1
    rc=$?; echo "count $C run $i exit $rc"; if fatal $rc; then exit $rc; fi
    grep '^{' gpurun_out/r4ae_c${C}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('   ', round(d['value'], 2), round(d['ms_per_step'], 2))"
  done
done
exit 0
