#!/bin/bash
# State machine with one-byte echo/ready entries (one root): the state-machine
# and sharded GPU tests, the state-machine round trace, and the default line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 600 python -u -m pytest tests/test_rbc_sim.py tests/test_sharded.py tests/test_broadcast_protocol.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3s8_tests.log 2>&1
rc=$?; echo "tests exit $rc"; tail -2 gpurun_out/r3s8_tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
HBRBC_JIT=load timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/r3s8_bench.log 2>&1
rc=$?; echo "bench exit $rc"; if fatal $rc; then exit $rc; fi
HBRBC_JIT=load TAG=r3s8 bash tools/gpu_sm_prof.sh > gpurun_out/r3s8_smprof.log 2>&1
echo "sm prof exit $?"
