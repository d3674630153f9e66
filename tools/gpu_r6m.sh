#!/bin/bash
# Round 6, call m: pairing kernels at 3 waves/SIMD (168 VGPRs, -DHB_PAIR_WPE=3,
# hbbft_amd/libhbrbc_w3.so) against the default 2, twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
  LIBS="libhbrbc.so libhbrbc_w3.so" bash tools/gpu_f4_ab.sh 2>&1 | grep -v "^W2026" | tee -a gpurun_out/r6m_f4_ab.txt
  rc=${PIPESTATUS[0]}; [ $rc -ne 0 ] && exit $rc
done
exit 0
