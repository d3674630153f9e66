#!/bin/bash
# Round 4, call c: the generic reconstruct's bit-pair form (HBRBC_GF=bitslice_pair)
# against the default, parity first, then alternating bench runs (instance
# mode, cfg3), then the pair form's issue counters.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_rbc_sim.py -m gpu -x -q --timeout 300 --timeout-method thread -k "gf_kernel_variants or single_root or matches_host or decode" > gpurun_out/r4c_gpu_tests.log 2>&1
rc=$?; echo "tests exit $rc"; tail -3 gpurun_out/r4c_gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for i in 1 2; do
  for G in bitslice bitslice_pair; do
    HBRBC_GF=$G HBRBC_JIT=load timeout -k 10 300 python bench.py --mode instances --steps 8 --warmup 2 --no-cpu --f4-checks 0 --no-leaf-reuse > gpurun_out/r4c_ab_${G}_$i.log 2>&1
    rc=$?; echo "ab $G $i exit $rc"; if fatal $rc; then exit $rc; fi
    grep '^{' gpurun_out/r4c_ab_${G}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('   ', d['value'], d['stages_ms_per_step']['reconstruct'])"
  done
done
HBRBC_GF=bitslice_pair TAG=r4c_gfpair CONFIG=cfg3 REGEX="gf_bitslice" \
SETS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA|SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_IFETCH SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE" \
  bash tools/pmc_stall.sh > /dev/null
rc=$?; echo "pmc exit $rc"; cat gpurun_out/pmc_r4c_gfpair/summary.txt
exit $rc
