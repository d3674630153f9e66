#!/bin/bash
# Round 3w: parity of the 7-row generic reconstruct (GPU parity tests), cfg5
# A/B of the specialised programs' LDS stage size and row tile, and cfg3 A/B
# of the generic kernel's inline set-bit path.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_unframe_fused.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3w_tests.log 2>&1
rc=$?; echo "tests exit $rc"; tail -2 gpurun_out/r3w_tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
export HBRBC_JIT=load
SETS="HBRBC_AB_BASE=1 HBRBC_JIT_LDS_STAGE=12 HBRBC_JIT_LDS_STAGE=16 HBRBC_JIT_LDS_STAGE=28 HBRBC_RT_SPEC=6 HBRBC_RT_SPEC=8 HBRBC_AB_BASE=2" CONFIGS=cfg5 STEPS=3 bash tools/ab_env.sh
rc=$?; echo "ab cfg5 exit $rc"; if fatal $rc; then exit $rc; fi
SETS="HBRBC_AB_BASE=1 HBRBC_GF=bitslice_likely HBRBC_AB_BASE=2 HBRBC_GF=bitslice_likely" CONFIGS=cfg3 STEPS=5 bash tools/ab_env.sh
rc=$?; echo "ab cfg3 exit $rc"
exit $rc
