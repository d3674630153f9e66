#!/bin/bash
# Round 4, call x: LDS stage size of the specialised programs at cfg5 (k = 84:
# default stages of 24 inputs), hiprtc-compiled on the box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp HBRBC_JIT=1
mkdir -p gpurun_out /tmp/jit_r4x
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
for L in 0 16 32 12; do
  if [ $L = 0 ]; then unset HBRBC_JIT_LDS_STAGE; else export HBRBC_JIT_LDS_STAGE=$L; fi
  HBRBC_JIT_DIR=/tmp/jit_r4x timeout -k 10 400 python bench.py --config cfg5 --mode instances --steps 6 --warmup 2 --no-cpu --f4-checks 0 --no-leaf-reuse > gpurun_out/r4x_lds${L}.log 2>&1
  rc=$?; echo "stage $L exit $rc"; if fatal $rc; then exit $rc; fi
  grep '^{' gpurun_out/r4x_lds${L}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); s=d['stages_ms_per_step']; print('   ', round(d['value'], 2), 'encode', round(s['encode'], 3), 'reconstruct', round(s['reconstruct'], 3))"
done
exit 0
