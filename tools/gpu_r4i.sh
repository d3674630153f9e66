#!/bin/bash
# Round 4, call i: global-records kernel read forms (constant address space,
# scalar mask words) on tools/sm_bench.py, then the full GPU suite, smoke and
# the default bench line on the default build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
for i in 1 2; do
  for L in a1u0 a1u1 a0u0; do
    HBRBC_JIT=load HBRBC_JIT_DIR=$PWD/hbbft_amd/jit HBRBC_LIB=$PWD/hbbft_amd/ab/libhbrbc_$L.so timeout -k 10 120 python tools/sm_bench.py --reps 7 >> gpurun_out/r4i_sm_ab.jsonl
    rc=$?; echo "sm $L exit $rc"; if fatal $rc; then exit $rc; fi
  done
done
cat gpurun_out/r4i_sm_ab.jsonl
TAG=r4i SKIP_REHEARSAL=1 BENCH_ARGS="--steps 10 --warmup 2" bash tools/gpu_round.sh
