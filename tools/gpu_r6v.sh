#!/bin/bash
# Round 6, call v: f4 with the cyclotomic square serialised too
# (HB_FP2_SERIAL=1, hbbft_amd/libhbrbc_cs.so) against the default, twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
  LIBS="libhbrbc.so libhbrbc_cs.so" bash tools/gpu_f4_ab.sh 2>&1 | grep -v "^W2026" | tee -a gpurun_out/r6v_f4_ab.txt
  rc=${PIPESTATUS[0]}; [ $rc -ne 0 ] && exit $rc
done
exit 0
