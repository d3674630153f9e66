#!/bin/bash
# Round 6, call aa: on the new default (serialised Fp2, f^|x| one unit):
# HB_FE_INL=1 (libhbrbc_efin.so) and HB_FP_CHAINS=1 (libhbrbc_ec1.so), and the whole Miller bit step as one unit (HB_MILLER_INL=3, libhbrbc_m3.so), twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
  LIBS="libhbrbc.so libhbrbc_efin.so libhbrbc_ec1.so libhbrbc_m3.so" bash tools/gpu_f4_ab.sh 2>&1 | grep -v "^W2026" | tee -a gpurun_out/r6aa_f4_ab.txt
  rc=${PIPESTATUS[0]}; [ $rc -ne 0 ] && exit $rc
done
exit 0
