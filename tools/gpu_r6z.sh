#!/bin/bash
# Round 6, call z: final-exponentiation inlining on the serialised-Fp2 base
# (HB_FE_INL=1 -> libhbrbc_sfin.so, HB_EXPX_INL=1 -> libhbrbc_sex1.so), twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
  LIBS="libhbrbc.so libhbrbc_sfin.so libhbrbc_sex1.so" bash tools/gpu_f4_ab.sh 2>&1 | grep -v "^W2026" | tee -a gpurun_out/r6z_f4_ab.txt
  rc=${PIPESTATUS[0]}; [ $rc -ne 0 ] && exit $rc
done
exit 0
