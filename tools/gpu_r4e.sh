#!/bin/bash
# Round 4, call e: state-machine A/B (register-cached mask word x merged
# Echo/EchoHash step, builds under hbbft_amd/ab/; 4-wave vs 3-wave forms) on
# tools/sm_bench.py, and the generic reconstruct at 3 vs 4 waves per block.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp HBRBC_JIT=load HBRBC_JIT_DIR=$PWD/hbbft_amd/jit
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
for W in auto 0; do
  for L in c0m0 c0m1 c1m0 c1m1; do
    if [ $W = auto ]; then unset HBRBC_SM_W4; else export HBRBC_SM_W4=$W; fi
    HBRBC_LIB=$PWD/hbbft_amd/ab/libhbrbc_$L.so timeout -k 10 120 python tools/sm_bench.py --reps 5 >> gpurun_out/r4e_sm_ab.jsonl 2> gpurun_out/r4e_sm_$L_$W.err
    rc=$?; echo "sm $L w4=$W exit $rc"; if fatal $rc; then exit $rc; fi
  done
done
unset HBRBC_SM_W4
cat gpurun_out/r4e_sm_ab.jsonl
for i in 1 2; do
  for NW in 4 3; do
    HBRBC_GF_WAVES=$NW timeout -k 10 300 python bench.py --mode instances --steps 8 --warmup 2 --no-cpu --f4-checks 0 --no-leaf-reuse > gpurun_out/r4e_gfw_${NW}_$i.log 2>&1
    rc=$?; echo "gf waves $NW $i exit $rc"; if fatal $rc; then exit $rc; fi
    grep '^{' gpurun_out/r4e_gfw_${NW}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('   ', d['value'], d['stages_ms_per_step']['reconstruct'])"
  done
done
exit 0
