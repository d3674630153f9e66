#!/bin/bash
# Round 6, call e: f4 Miller-step inlining A/B (HB_MILLER_INL 0 / 1 / 2 as
# hbbft_amd/libhbrbc{,_mi1,_mi2}.so), pairing parity per build, then the
# grouped-check kernels' times under a kernel trace, twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
  LIBS="libhbrbc.so libhbrbc_mi1.so libhbrbc_mi2.so" bash tools/gpu_f4_ab.sh 2>&1 | tee -a gpurun_out/r6e_f4_ab.txt
  rc=${PIPESTATUS[0]}; [ $rc -ne 0 ] && exit $rc
done
exit 0
