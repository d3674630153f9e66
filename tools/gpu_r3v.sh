#!/bin/bash
# Round-3 validation: every GPU test, smoke, then cfg3 kernel trace/stats +
# PMC traffic passes of the default code, then the default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3v_tests.log 2>&1
rc=$?; echo "tests exit $rc"; tail -2 gpurun_out/r3v_tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3v_smoke.log 2>&1
rc=$?; echo "smoke exit $rc"; if [ $rc -ne 0 ]; then exit $rc; fi
export HBRBC_JIT=load
TAG=r3v BENCH_ARGS="--steps 5 --warmup 1 --no-cpu --mode instances --f4-checks 0" PMC_ARGS="--steps 1 --warmup 1 --no-cpu --mode instances --no-verify --f4-checks 0" bash tools/profile.sh > gpurun_out/r3v_profile.log 2>&1
rc=$?; echo "profile exit $rc"; if fatal $rc; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/r3v_bench.log 2>&1
rc=$?; echo "bench exit $rc"; if fatal $rc; then exit $rc; fi
# A/B: generic reconstruct row tile 6 (default at N=64: passes 6,6,6,3) vs 7 (7,7,7)
for r in 7 6; do
  HBRBC_RT_REC=$r timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu --mode instances --f4-checks 0 > gpurun_out/r3v_rt$r.log 2>&1
  rc=$?; echo "rt $r exit $rc"; if fatal $rc; then exit $rc; fi
done
# instruction-cache counters of the GF kernels (large straight-line XOR networks)
for c in cfg5 cfg3; do
  TAG=r3v_icache_$c CONFIG=$c SETS="SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU" bash tools/pmc_stall.sh > gpurun_out/r3v_icache_$c.log 2>&1
  rc=$?; echo "icache $c exit $rc"; if [ $rc -ne 0 ]; then exit $rc; fi
done
