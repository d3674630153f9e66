#!/bin/bash
# Round 4, call d = calls b + c in one box lease (the pool is contended):
# parity (GF forms incl. bit pairs, state machine incl. the merged Echo /
# EchoHash step, sharded, footprint), the instance-mode bench, GF counters of
# both forms, state-machine counters at N=128, the GF form A/B, and the
# pair-lane rebuilt-row leaf hash A/B in validator mode.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_unframe_fused.py tests/test_sharded.py tests/test_layouts.py tests/test_rbc_sim.py tests/test_broadcast_protocol.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4d_gpu_tests.log 2>&1
rc=$?; echo "tests exit $rc"; tail -3 gpurun_out/r4d_gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
HBRBC_JIT=load timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --f4-checks 0 > gpurun_out/r4d_bench.log 2>&1
rc=$?; echo "bench exit $rc"; if fatal $rc; then exit $rc; fi
grep '^{' gpurun_out/r4d_bench.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('   head', d['value'], {k: round(v, 3) for k, v in d['stages_ms_per_step'].items()})
print('   leaf_reuse', d['leaf_reuse']['value'])
for o in ('validators', 'validators_cfg4'): print('  ', o, d[o].get('value'), {k: round(v, 3) for k, v in d[o].get('stages_ms_per_step', {}).items()})"
for i in 1 2; do
  for G in bitslice bitslice_pair; do
    HBRBC_GF=$G HBRBC_JIT=load timeout -k 10 300 python bench.py --mode instances --steps 8 --warmup 2 --no-cpu --f4-checks 0 --no-leaf-reuse > gpurun_out/r4d_ab_${G}_$i.log 2>&1
    rc=$?; echo "ab $G $i exit $rc"; if fatal $rc; then exit $rc; fi
    grep '^{' gpurun_out/r4d_ab_${G}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('   ', d['value'], d['stages_ms_per_step']['reconstruct'])"
  done
done
for G in bitslice bitslice_pair; do
  HBRBC_GF=$G TAG=r4d_gf_$G CONFIG=cfg3 REGEX="gf_bitslice" \
  SETS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA|SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_IFETCH SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE" \
    bash tools/pmc_stall.sh > /dev/null
  rc=$?; echo "pmc gf $G exit $rc"; cat gpurun_out/pmc_r4d_gf_$G/summary.txt; if fatal $rc; then exit $rc; fi
done
MODE=validators TAG=r4d_sm CONFIG=cfg4 REGEX="sm_round" \
SETS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS|SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_LDS_BANK_CONFLICT|SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_IFETCH GRBM_GUI_ACTIVE" \
  bash tools/pmc_stall.sh > /dev/null
rc=$?; echo "pmc sm exit $rc"; cat gpurun_out/pmc_r4d_sm/summary.txt; if fatal $rc; then exit $rc; fi
OUT=$PWD/gpurun_out/prof_r4d_sm; mkdir -p $OUT
HBRBC_JIT=load timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 bench.py --mode validators --config cfg4 --steps 5 --warmup 1 --no-cpu --f4-checks 0 > $OUT/trace.log 2>&1
rc=$?; echo "sm trace exit $rc"; if fatal $rc; then exit $rc; fi
for PB in 0 262144; do
  HBRBC_LIST_PAIR_BELOW=$PB HBRBC_JIT=load timeout -k 10 300 python bench.py --mode validators --steps 8 --warmup 2 --no-cpu --f4-checks 0 > gpurun_out/r4d_vpair_$PB.log 2>&1
  rc=$?; echo "vpair $PB exit $rc"; if fatal $rc; then exit $rc; fi
  grep '^{' gpurun_out/r4d_vpair_$PB.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['validators']; print('   ', d['value'], d['stages_ms_per_step']['leaf_hash'])"
done
exit 0
