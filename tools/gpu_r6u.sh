#!/bin/bash
# Round 6, call u: f4 with serialised Fp products in every Fp2 product
# (HB_FP2_SERIAL=1, hbbft_amd/libhbrbc_fs.so) against the default, twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
  LIBS="libhbrbc.so libhbrbc_fs.so" bash tools/gpu_f4_ab.sh 2>&1 | grep -v "^W2026" | tee -a gpurun_out/r6u_f4_ab.txt
  rc=${PIPESTATUS[0]}; [ $rc -ne 0 ] && exit $rc
done
exit 0
