#!/bin/bash
# Round 6, call g: final-exponentiation A/B (HB_FE_INL / HB_FE_WPE builds
# hbbft_amd/libhbrbc_{fin,fw1,fw1in}.so; default = Miller steps inlined),
# then the own-stream pipelines A/B and the 4-rank rehearsal (tools/gpu_r6f.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
LIBS="libhbrbc.so libhbrbc_fin.so libhbrbc_fw1.so libhbrbc_fw1in.so" bash tools/gpu_f4_ab.sh 2>&1 | tee gpurun_out/r6g_f4_ab.txt
rc=${PIPESTATUS[0]}; [ $rc -ne 0 ] && exit $rc
unset HBRBC_LIB
bash tools/gpu_r6f.sh
