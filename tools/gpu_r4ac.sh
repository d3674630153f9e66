#!/bin/bash
# Round 4, call ac: instances per step of the other instance configs
# (cfg2 4096 / 16384, cfg4 8192 / 16384, cfg5 1024 / 2048).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp HBRBC_JIT=load
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
for V in cfg2:4096 cfg2:16384 cfg4:8192 cfg4:16384 cfg5:1024 cfg5:2048; do
  C=${V%%:*}; N=${V#*:}
  timeout -k 10 400 python bench.py --config $C --mode instances --count $N --steps 5 --warmup 2 --no-cpu --f4-checks 0 --no-leaf-reuse > gpurun_out/r4ac_${C}_$N.log 2>&1
  rc=$?; echo "$C count $N exit $rc"; if fatal $rc; then exit $rc; fi
  grep '^{' gpurun_out/r4ac_${C}_$N.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); s=d['stages_ms_per_step']; print('   ', round(d['value'], 2), round(d['ms_per_step'], 2), {k: round(v, 2) for k, v in s.items() if v > 0.5})"
done
exit 0
