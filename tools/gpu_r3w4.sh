#!/bin/bash
# A/B: state-machine round kernels at 4 waves/SIMD (128 VGPRs, some spills)
# against the default (162 VGPRs, 3 waves/SIMD): validator-sharded objects.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 HBRBC_JIT=load
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
for v in base w4 base w4; do
  if [ $v = w4 ]; then L=$PWD/hbbft_amd/libhbrbc_smw4.so; else L=$PWD/hbbft_amd/libhbrbc.so; fi
  HBRBC_LIB=$L timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu --f4-checks 0 > gpurun_out/r3w4_$v.log 2>&1
  rc=$?; echo "$v exit $rc"; if fatal $rc; then exit $rc; fi
  tail -1 gpurun_out/r3w4_$v.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); v=d['validators']; v4=d['validators_cfg4']
print('$v', round(v['value'],2), round(v['stages_ms_per_step']['state_machine'],3), round(v4['value'],2), round(v4['stages_ms_per_step']['state_machine'],3))"
done
