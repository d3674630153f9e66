#!/bin/bash
# Round 4, call m: the generic reconstruct with input pairs per step
# (HBRBC_GF=bitslice_x2, one v_xor3 folds both inputs' multiples): parity,
# instance-mode A/B against the one-input form (default lib, 3 waves/SIMD at
# 135 VGPRs; ab/libhbrbc_gfw4.so, register budget cut to 4 waves), counters.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_unframe_fused.py -m gpu -x -q --timeout 240 --timeout-method thread -k "variants or unframe" > gpurun_out/r4m_tests.log 2>&1
rc=$?; echo "tests exit $rc"; tail -3 gpurun_out/r4m_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
export HBRBC_JIT=load
for i in 1 2; do
  for V in bitslice:libhbrbc.so bitslice_x2:libhbrbc.so bitslice_x2:ab/libhbrbc_gfw4.so; do
    G=${V%%:*}; L=${V#*:}; T=${G}_$(basename $L .so)_$i
    HBRBC_GF=$G HBRBC_LIB=$PWD/hbbft_amd/$L timeout -k 10 300 python bench.py --mode instances --steps 8 --warmup 2 --no-cpu --f4-checks 0 --no-leaf-reuse > gpurun_out/r4m_ab_$T.log 2>&1
    rc=$?; echo "ab $T exit $rc"; if fatal $rc; then exit $rc; fi
    grep '^{' gpurun_out/r4m_ab_$T.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('   ', round(d['value'], 2), round(d['stages_ms_per_step']['reconstruct'], 3))"
  done
done
HBRBC_GF=bitslice_x2 TAG=r4m_gf_x2 CONFIG=cfg3 REGEX="gf_bitslice" \
SETS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA|SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_IFETCH SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE" \
  bash tools/pmc_stall.sh > /dev/null
rc=$?; echo "pmc exit $rc"; cat gpurun_out/pmc_r4m_gf_x2/summary.txt
exit $rc
