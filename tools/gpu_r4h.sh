#!/bin/bash
# Round 4, call h: the state machine with scalar record reads in the
# global-records kernel (parity, then records through LDS vs global memory on
# tools/sm_bench.py), then the committed cfg3 profile set (tools/gpu_r4f.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 600 python -u -m pytest tests/test_rbc_sim.py tests/test_sharded.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4h_gpu_tests.log 2>&1
rc=$?; echo "tests exit $rc"; tail -3 gpurun_out/r4h_gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for i in 1 2; do
  for G in 1 0; do
    HBRBC_JIT=load HBRBC_SM_GREC=$G timeout -k 10 120 python tools/sm_bench.py --reps 7 | sed "s/}$/, \"grec\": $G}/" >> gpurun_out/r4h_sm_ab.jsonl
    rc=$?; echo "sm grec=$G exit $rc"; if fatal $rc; then exit $rc; fi
  done
done
cat gpurun_out/r4h_sm_ab.jsonl
bash tools/gpu_r4f.sh
