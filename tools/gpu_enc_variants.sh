#!/bin/bash
# cfg3 encoder A/B (instance mode only): streaming vs LDS-staged XOR networks.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 HBRBC_JIT=load
mkdir -p gpurun_out
VARIANTS="${VARIANTS:-HBRBC_JIT_LDS=0 --mode instances --f4-checks 0;HBRBC_JIT_LDS=1 HBRBC_JIT_LDS_STAGE=22 HBRBC_JIT_NET=2 --mode instances --f4-checks 0;HBRBC_JIT_LDS=1 HBRBC_RT_SPEC=11 HBRBC_JIT_LDS_STAGE=22 HBRBC_JIT_NET=2 HBRBC_JIT_WPE=3 --mode instances --f4-checks 0;HBRBC_JIT_LDS=1 HBRBC_RT_SPEC=11 HBRBC_JIT_LDS_STAGE=22 HBRBC_JIT_NET=1 HBRBC_JIT_WPE=3 --mode instances --f4-checks 0;HBRBC_JIT_LDS=1 HBRBC_RT_SPEC=7 HBRBC_JIT_LDS_STAGE=22 HBRBC_JIT_NET=2 HBRBC_JIT_WPE=4 --mode instances --f4-checks 0;HBRBC_JIT_LDS=1 HBRBC_RT_SPEC=7 HBRBC_JIT_LDS_STAGE=22 HBRBC_JIT_NET=1 HBRBC_JIT_WPE=4 --mode instances --f4-checks 0}" bash tools/bench_variants.sh 2>&1 | tee gpurun_out/enc_variants.txt
