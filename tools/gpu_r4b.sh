#!/bin/bash
# Round 4, call b: parity of the generic GF kernel with scalar-operand
# prefetch, its counters (incl. branches / instruction fetch), the state
# machine's counters at N=128, a bench of the instance mode, and the pair-lane
# rebuilt-row leaf hash A/B in validator mode.  Stops at the first fatal status.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_unframe_fused.py tests/test_sharded.py tests/test_layouts.py tests/test_rbc_sim.py tests/test_broadcast_protocol.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4b_gpu_tests.log 2>&1
rc=$?; echo "tests exit $rc"; tail -3 gpurun_out/r4b_gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
HBRBC_JIT=load timeout -k 10 300 python bench.py --mode instances --steps 10 --warmup 2 --no-cpu --f4-checks 0 > gpurun_out/r4b_bench_inst.log 2>&1
rc=$?; echo "bench inst exit $rc"; if fatal $rc; then exit $rc; fi
TAG=r4b_gf CONFIG=cfg3 REGEX="gf_bitslice" \
SETS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA|SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_IFETCH SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE" \
  bash tools/pmc_stall.sh > /dev/null
rc=$?; echo "pmc gf exit $rc"; cat gpurun_out/pmc_r4b_gf/summary.txt; if fatal $rc; then exit $rc; fi
MODE=validators TAG=r4b_sm CONFIG=cfg4 REGEX="sm_round" \
SETS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS|SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_LDS_BANK_CONFLICT|SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_IFETCH GRBM_GUI_ACTIVE" \
  bash tools/pmc_stall.sh > /dev/null
rc=$?; echo "pmc sm exit $rc"; cat gpurun_out/pmc_r4b_sm/summary.txt; if fatal $rc; then exit $rc; fi
for PB in 0 262144; do
  HBRBC_LIST_PAIR_BELOW=$PB HBRBC_JIT=load timeout -k 10 300 python bench.py --mode validators --steps 8 --warmup 2 --no-cpu --f4-checks 0 > gpurun_out/r4b_vpair_$PB.log 2>&1
  rc=$?; echo "vpair $PB exit $rc"; if fatal $rc; then exit $rc; fi
done
exit 0
