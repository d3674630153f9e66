#!/bin/bash
# Round 6, call j: exp-by-x inlining A/B (HB_EXPX_INL / HB_FE_INL builds
# hbbft_amd/libhbrbc_{ex1,ex1fin}.so against the default), twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
  LIBS="libhbrbc.so libhbrbc_ex1.so libhbrbc_ex1fin.so" bash tools/gpu_f4_ab.sh 2>&1 | grep -v "^W2026" | tee -a gpurun_out/r6j_f4_ab.txt
  rc=${PIPESTATUS[0]}; [ $rc -ne 0 ] && exit $rc
done
exit 0
