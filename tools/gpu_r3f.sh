#!/bin/bash
# Round-3 final: cfg3 kernel trace/stats + PMC passes of the final code, then
# the default line and the 2-rank gloo rehearsal (tools/gpu_round.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
HBRBC_JIT=load TAG=r3f BENCH_ARGS="--steps 5 --warmup 1 --no-cpu --mode instances --f4-checks 0" PMC_ARGS="--steps 1 --warmup 1 --no-cpu --mode instances --no-verify --f4-checks 0" bash tools/profile.sh > gpurun_out/r3f_profile.log 2>&1
rc=$?; echo "profile exit $rc"; if fatal $rc; then exit $rc; fi
# two sub-batches on two streams (re-measured now that encode / reconstruct are
# closer to HBM-bound than VALU-bound)
for ns in "2" "2 --stagger" "4 --stagger" "1"; do
  tag=$(echo "$ns" | tr -d ' -')
  HBRBC_JIT=load timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu --mode instances --f4-checks 0 --streams $ns > gpurun_out/r3f_streams$tag.log 2>&1
  rc=$?; echo "streams $ns exit $rc"; if fatal $rc; then exit $rc; fi
done
SKIP_TESTS=1 TAG=r3f bash tools/gpu_round.sh
