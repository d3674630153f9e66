#!/bin/bash
# Round 4, call k: the other instance configs (cfg2, cfg4, cfg5) on the
# round-4 code, and the 2-rank gloo rehearsal of the multi-GPU line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp HBRBC_JIT=load
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
for C in cfg4 cfg5 cfg2; do
  timeout -k 10 400 python bench.py --config $C --mode instances --steps 8 --warmup 2 --f4-checks 0 --cpu-reps 3 > gpurun_out/r4k_$C.log 2>&1
  rc=$?; echo "$C exit $rc"; if fatal $rc; then exit $rc; fi
  grep '^{' gpurun_out/r4k_$C.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('   ', round(d['value'], 2), round(d['ms_per_step'], 2), {k: round(v, 2) for k, v in d['stages_ms_per_step'].items()}, 'cpu', d['cpu_baseline'] and round(d['cpu_baseline']['value'], 3))"
done
HBRBC_BENCH_REHEARSE=1 timeout -k 10 600 python bench.py --gpus 2 --steps 3 --warmup 1 --f4-checks 65536 > gpurun_out/r4k_rehearsal_g2.log 2>&1
rc=$?; echo "rehearsal exit $rc"; tail -c 600 gpurun_out/r4k_rehearsal_g2.log
exit $rc
