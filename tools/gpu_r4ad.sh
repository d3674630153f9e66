#!/bin/bash
# Round 4, call ad: cfg2 at BASELINE's batch of 4096 instances with 1 / 2 / 4
# batches in flight on their own streams (--streams k --count 4096 k), and
# the cfg4 / cfg5 instance lines at their new defaults with the CPU baseline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp HBRBC_JIT=load
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
for K in 1 2 4; do
  timeout -k 10 400 python bench.py --config cfg2 --mode instances --count $((4096 * K)) --streams $K --steps 5 --warmup 2 --no-cpu --f4-checks 0 --no-leaf-reuse > gpurun_out/r4ad_cfg2_s$K.log 2>&1
  rc=$?; echo "cfg2 streams $K exit $rc"; if fatal $rc; then exit $rc; fi
  grep '^{' gpurun_out/r4ad_cfg2_s$K.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('   ', round(d['value'], 2), round(d['ms_per_step'], 2))"
done
for C in cfg4 cfg5; do
  timeout -k 10 500 python bench.py --config $C --mode instances --steps 6 --warmup 2 --f4-checks 0 --cpu-reps 3 > gpurun_out/r4ad_$C.log 2>&1
  rc=$?; echo "$C exit $rc"; if fatal $rc; then exit $rc; fi
  grep '^{' gpurun_out/r4ad_$C.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('   ', round(d['value'], 2), round(d['ms_per_step'], 2), 'cpu', d['cpu_baseline'] and round(d['cpu_baseline']['value'], 3))"
done
exit 0
