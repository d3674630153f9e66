#!/bin/bash
# Round 6, call x: f4 at 3 waves per SIMD on the serialised Fp2 product
# (HB_FP2_SERIAL=1, hbbft_amd/libhbrbc_sw3.so) against the default, twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
  LIBS="libhbrbc.so libhbrbc_sw3.so" bash tools/gpu_f4_ab.sh 2>&1 | grep -v "^W2026" | tee -a gpurun_out/r6x_f4_ab.txt
  rc=${PIPESTATUS[0]}; [ $rc -ne 0 ] && exit $rc
done
exit 0
