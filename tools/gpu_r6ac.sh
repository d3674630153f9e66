#!/bin/bash
# Round 6, call ac: the Miller-step inlining levels on the final base:
# HB_MILLER_INL=1 (libhbrbc_mi1.so) and 0 (libhbrbc_mi0.so) against the default 2, and the G2 line units without the serialisation (HB_G2_SERIAL=0, libhbrbc_g2p.so), twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
  LIBS="libhbrbc.so libhbrbc_mi1.so libhbrbc_mi0.so libhbrbc_g2p.so" bash tools/gpu_f4_ab.sh 2>&1 | grep -v "^W2026" | tee -a gpurun_out/r6ac_f4_ab.txt
  rc=${PIPESTATUS[0]}; [ $rc -ne 0 ] && exit $rc
done
exit 0
