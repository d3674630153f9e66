#!/bin/bash
# Round 4, call g: parity of the global-records state-machine kernels and the
# balanced GF waves, then the state machine's launch forms on
# tools/sm_bench.py (records through LDS or global memory x 4 / 3 waves per
# SIMD), then the f4 product-scanning chain count A/B (tools/gpu_f4_ab.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 600 python -u -m pytest tests/test_rbc_sim.py tests/test_sharded.py tests/test_gpu_parity.py tests/test_unframe_fused.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4g_gpu_tests.log 2>&1
rc=$?; echo "tests exit $rc"; tail -3 gpurun_out/r4g_gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for G in 1 0; do
  for W in auto 0 1; do
    if [ $W = auto ]; then unset HBRBC_SM_W4; else export HBRBC_SM_W4=$W; fi
    HBRBC_JIT=load HBRBC_SM_GREC=$G timeout -k 10 120 python tools/sm_bench.py --reps 5 | sed "s/}$/, \"grec\": $G}/" >> gpurun_out/r4g_sm_ab.jsonl
    rc=$?; echo "sm grec=$G w4=$W exit $rc"; if fatal $rc; then exit $rc; fi
  done
done
unset HBRBC_SM_W4
cat gpurun_out/r4g_sm_ab.jsonl
for i in 1 2; do
  for V in "" "HBRBC_RT_SPEC=11" "HBRBC_RT_SPEC=11 HBRBC_JIT_WPE=4" "HBRBC_RT_SPEC=14"; do
    env $V HBRBC_JIT=load timeout -k 10 120 python tools/enc_bench.py >> gpurun_out/r4g_enc_ab.jsonl
    rc=$?; echo "enc [$V] exit $rc"; if fatal $rc; then exit $rc; fi
  done
done
cat gpurun_out/r4g_enc_ab.jsonl
LIBS="libhbrbc.so ab/libhbrbc_fp4.so" bash tools/gpu_f4_ab.sh
rc=$?; echo "f4 ab exit $rc"
exit $rc
