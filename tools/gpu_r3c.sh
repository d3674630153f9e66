#!/bin/bash
# Round 3c: tests + smoke on the new defaults, the default bench line, the
# other configs' instance lines, and the rocprofv3 passes of the cfg3 line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r3c_gpu_tests.log 2>&1
rc=$?; echo "tests exit $rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r3c_gpu_tests.log | tail -12
if fatal $rc; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3c_smoke.log 2>&1
rc=$?; echo "smoke exit $rc"; tail -2 gpurun_out/r3c_smoke.log
if fatal $rc; then exit $rc; fi
export HBRBC_JIT=load
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/r3c_bench.log 2>&1
rc=$?; echo "bench exit $rc"; if fatal $rc; then exit $rc; fi
for c in cfg2 cfg4 cfg5; do
  timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 1 --f4-checks 0 --cpu-seconds 2 > gpurun_out/r3c_bench_$c.log 2>&1
  rc=$?; echo "bench $c exit $rc"; if fatal $rc; then exit $rc; fi
done
TAG=r3c BENCH_ARGS="--steps 5 --warmup 1 --no-cpu --mode instances --f4-checks 0" PMC_ARGS="--steps 1 --warmup 1 --no-cpu --mode instances --no-verify --f4-checks 0" bash tools/profile.sh
