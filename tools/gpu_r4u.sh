#!/bin/bash
# Round 4, call u: LDS stage size of the specialised encoder at cfg3
# (HBRBC_JIT_LDS_STAGE: inputs per LDS stage; default = all 22 in one stage).
# Variant code objects are compiled by hiprtc on the box (not cached).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp HBRBC_JIT=1
mkdir -p gpurun_out /tmp/jit_r4u
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
for i in 1 2; do
  for L in 0 11 8 6; do
    if [ $L = 0 ]; then unset HBRBC_JIT_LDS_STAGE; else export HBRBC_JIT_LDS_STAGE=$L; fi
    HBRBC_JIT_DIR=/tmp/jit_r4u timeout -k 10 300 python bench.py --mode instances --steps 8 --warmup 2 --no-cpu --f4-checks 0 --no-leaf-reuse > gpurun_out/r4u_lds${L}_$i.log 2>&1
    rc=$?; echo "stage $L run $i exit $rc"; if fatal $rc; then exit $rc; fi
    grep '^{' gpurun_out/r4u_lds${L}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('   ', round(d['value'], 2), round(d['stages_ms_per_step']['encode'], 3))"
  done
done
exit 0
