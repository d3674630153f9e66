#!/bin/bash
# Round 4, call aj: cfg3 instance mode at 32768 instances split over 1 / 2 / 4
# sub-batches on their own streams (plain and staggered).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp HBRBC_JIT=load
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
for V in 1: 2: 4: 2:--stagger 4:--stagger; do
  K=${V%%:*}; X=${V#*:}
  T=s${K}$( [ -n "$X" ] && echo _stag )
  timeout -k 10 400 python bench.py --mode instances --streams $K $X --steps 6 --warmup 2 --no-cpu --f4-checks 0 --no-leaf-reuse > gpurun_out/r4aj_$T.log 2>&1
  rc=$?; echo "$T exit $rc"; if fatal $rc; then exit $rc; fi
  grep '^{' gpurun_out/r4aj_$T.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('   ', round(d['value'], 2), round(d['ms_per_step'], 2), round(d['stages_ms_per_step']['leaf_hash'], 1))"
done
exit 0
