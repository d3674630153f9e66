#!/bin/bash
# Round-3 A/B on one box: cfg3 encoder forms (streaming vs LDS-staged), then
# cfg5 with the N = 250 programs serial vs concurrent (HBRBC_XOR_STREAMS).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 HBRBC_JIT=load
mkdir -p gpurun_out
bash tools/gpu_enc_variants.sh
rc=$?; case $rc in 124|134|137|139) exit $rc;; esac
VARIANTS="HBRBC_XOR_STREAMS=0 --config cfg5 --mode instances --f4-checks 0;HBRBC_XOR_STREAMS=1 --config cfg5 --mode instances --f4-checks 0" bash tools/bench_variants.sh 2>&1 | tee gpurun_out/cfg5_streams.txt
