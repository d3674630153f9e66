#!/bin/bash
# Round 3b: full GPU tests with the LDS-form defaults, pair-lane sponge
# parity, then A/B: cfg4 / cfg5 LDS form, pair-lane sponges (cfg2 leaf
# hash, per-call validate).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r3b_gpu_tests.log 2>&1
rc=$?; echo "tests exit $rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r3b_gpu_tests.log | tail -12
if fatal $rc; then exit $rc; fi
HBRBC_SPONGE_PAIR=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_layouts.py tests/test_unframe_fused.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r3b_pair_tests.log 2>&1
rc=$?; echo "pair-lane tests exit $rc"; tail -3 gpurun_out/r3b_pair_tests.log
if fatal $rc; then exit $rc; fi
export HBRBC_JIT=load
VARIANTS="--mode instances --f4-checks 0;HBRBC_JIT_LDS=0 --mode instances --f4-checks 0;--config cfg4 --mode instances --f4-checks 0;HBRBC_JIT_LDS=1 HBRBC_RT_SPEC=11 HBRBC_JIT_WPE=3 --config cfg4 --mode instances --f4-checks 0;--config cfg5 --mode instances --f4-checks 0;HBRBC_JIT_LDS=1 HBRBC_RT_SPEC=7 HBRBC_JIT_WPE=4 --config cfg5 --mode instances --f4-checks 0;--config cfg2 --mode instances --f4-checks 0;HBRBC_SPONGE_PAIR=2 --config cfg2 --mode instances --f4-checks 0" bash tools/bench_variants.sh 2>&1 | tee gpurun_out/r3b_variants.txt
rc=${PIPESTATUS[0]}; if fatal $rc; then exit $rc; fi
timeout -k 10 300 python tools/bench_percall.py gpurun_out/r3b_percall_single.jsonl > /dev/null 2>&1; echo "percall exit $?"
HBRBC_SPONGE_PAIR=1 timeout -k 10 300 python tools/bench_percall.py gpurun_out/r3b_percall_pair.jsonl > /dev/null 2>&1; echo "percall pair exit $?"
