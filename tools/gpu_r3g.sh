#!/bin/bash
# Round-3 profiles: cfg3 kernel trace/stats + PMC traffic and VALU passes,
# cfg3 stall counters, the same for cfg5, and the cfg5 / cfg2 / cfg4 bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 HBRBC_JIT=load
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
TAG=r3 BENCH_ARGS="--steps 5 --warmup 1 --no-cpu --mode instances --f4-checks 0" PMC_ARGS="--steps 1 --warmup 1 --no-cpu --mode instances --no-verify --f4-checks 0" bash tools/profile.sh
rc=$?; echo "profile cfg3 exit $rc"; if fatal $rc; then exit $rc; fi
TAG=r3_cfg5 BENCH_ARGS="--config cfg5 --steps 3 --warmup 1 --no-cpu --mode instances --f4-checks 0" PMC_ARGS="--config cfg5 --steps 1 --warmup 1 --no-cpu --mode instances --no-verify --f4-checks 0" bash tools/profile.sh
rc=$?; echo "profile cfg5 exit $rc"; if fatal $rc; then exit $rc; fi
TAG=r3_stall CONFIG=cfg3 bash tools/pmc_stall.sh > /dev/null
rc=$?; echo "stall cfg3 exit $rc"; if fatal $rc; then exit $rc; fi
for c in cfg5 cfg2 cfg4; do
  timeout -k 10 400 python bench.py --config $c --steps 5 --warmup 1 --f4-checks 0 --mode instances --cpu-seconds 2 --cpu-reps 3 > gpurun_out/r3g_bench_$c.log 2>&1
  rc=$?; echo "bench $c exit $rc"; if fatal $rc; then exit $rc; fi
done
