#!/bin/bash
# Round 3x: every GPU test with the 6-row split programs (N = 250) and 7-row
# generic reconstruct (N = 64), cfg5 bench line + profile, default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3x_tests.log 2>&1
rc=$?; echo "tests exit $rc"; tail -2 gpurun_out/r3x_tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
export HBRBC_JIT=load
timeout -k 10 400 python bench.py --config cfg5 --steps 5 --warmup 1 --f4-checks 0 --mode instances --cpu-seconds 2 --cpu-reps 3 > gpurun_out/r3x_bench_cfg5.log 2>&1
rc=$?; echo "bench cfg5 exit $rc"; if fatal $rc; then exit $rc; fi
TAG=r3x_cfg5 BENCH_ARGS="--config cfg5 --steps 3 --warmup 1 --no-cpu --mode instances --f4-checks 0" PMC_ARGS="--config cfg5 --steps 1 --warmup 1 --no-cpu --mode instances --no-verify --f4-checks 0" bash tools/profile.sh > gpurun_out/r3x_profile_cfg5.log 2>&1
rc=$?; echo "profile cfg5 exit $rc"; if fatal $rc; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/r3x_bench.log 2>&1
rc=$?; echo "bench exit $rc"
exit $rc
