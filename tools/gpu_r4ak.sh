#!/bin/bash
# Round 4, call ak: hardware queues per process (GPU_MAX_HW_QUEUES 4 default vs
# 8) under the validator line's streams (two step pipelines, each with a side
# stream) and cfg3 with 2 sub-batch streams.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp HBRBC_JIT=load
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
for i in 1 2; do
  for Q in 4 8; do
    GPU_MAX_HW_QUEUES=$Q timeout -k 10 300 python bench.py --mode validators --steps 10 --warmup 2 --no-cpu --f4-checks 0 > gpurun_out/r4ak_v_q${Q}_$i.log 2>&1
    rc=$?; echo "validators queues $Q run $i exit $rc"; if fatal $rc; then exit $rc; fi
    grep '^{' gpurun_out/r4ak_v_q${Q}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['validators']; print('   ', round(d['value'], 2), round(d['ms_per_step'], 3))"
  done
done
for Q in 4 8; do
  GPU_MAX_HW_QUEUES=$Q timeout -k 10 400 python bench.py --mode instances --streams 2 --steps 6 --warmup 2 --no-cpu --f4-checks 0 --no-leaf-reuse > gpurun_out/r4ak_s2_q$Q.log 2>&1
  rc=$?; echo "cfg3 streams 2 queues $Q exit $rc"; if fatal $rc; then exit $rc; fi
  grep '^{' gpurun_out/r4ak_s2_q$Q.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('   ', round(d['value'], 2), round(d['ms_per_step'], 2), round(d['stages_ms_per_step']['leaf_hash'], 1))"
done
exit 0
