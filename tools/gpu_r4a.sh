#!/bin/bash
# Round 4, first GPU call: the GPU suite (with the single-root state-machine
# parity cases), then the issue/stall counters of the generic reconstruct
# kernel gf_bitslice_kernel<7,0> at cfg3 (one rocprofv3 --pmc pass per group),
# and the counter list of this rocprofv3.  Stops at the first fatal status.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/r4a_gpu_tests.log 2>&1
  rc=$?; echo "tests exit $rc"; tail -4 gpurun_out/r4a_gpu_tests.log
  if fatal $rc; then exit $rc; fi
fi
timeout -k 10 60 rocprofv3 -L > gpurun_out/r4a_counters.txt 2>&1; echo "list exit $?"
TAG=r4a_gf CONFIG=cfg3 REGEX="gf_bitslice" \
SETS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA|SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE" \
  bash tools/pmc_stall.sh
rc=$?; echo "pmc exit $rc"
if fatal $rc; then exit $rc; fi
# the default line (leaf_reuse variant, validator objects with the new
# state-machine entries) under a kernel trace
OUT=$PWD/gpurun_out/prof_r4a
mkdir -p $OUT
HBRBC_JIT=load timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu --f4-checks 0 > gpurun_out/r4a_bench.log 2>&1
rc=$?; echo "bench exit $rc"; tail -c 600 gpurun_out/r4a_bench.log
exit $rc
