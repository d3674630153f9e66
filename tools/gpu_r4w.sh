#!/bin/bash
# Round 4, call w: the global-records state-machine kernel with each sender's
# inbox slot prefetched one sender ahead (HB_SM_PF=1, default build) against
# the dependent-load loop (ab/libhbrbc_pf0.so): per-node parity of the state
# machine, tools/sm_bench.py, validator cfg4 line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 600 python -u -m pytest tests/test_rbc_sim.py tests/test_sharded.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4w_tests.log 2>&1
rc=$?; echo "tests exit $rc"; tail -2 gpurun_out/r4w_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
export HBRBC_JIT=load HBRBC_JIT_DIR=$PWD/hbbft_amd/jit
for i in 1 2; do
  for L in libhbrbc.so ab/libhbrbc_pf0.so; do
    HBRBC_LIB=$PWD/hbbft_amd/$L timeout -k 10 120 python tools/sm_bench.py --reps 7 >> gpurun_out/r4w_sm_ab.jsonl
    rc=$?; echo "sm $L exit $rc"; if fatal $rc; then exit $rc; fi
  done
done
cat gpurun_out/r4w_sm_ab.jsonl
export HBRBC_JIT=load HBRBC_JIT_DIR=$PWD/hbbft_amd/jit
for i in 1 2; do
  for L in libhbrbc.so ab/libhbrbc_pf0.so; do
    T=$(basename $L .so)_$i
    HBRBC_LIB=$PWD/hbbft_amd/$L timeout -k 10 300 python bench.py --mode validators --config cfg4 --steps 12 --warmup 2 --no-cpu --f4-checks 0 > gpurun_out/r4w_cfg4_$T.log 2>&1
    rc=$?; echo "cfg4 $T exit $rc"; if fatal $rc; then exit $rc; fi
    grep '^{' gpurun_out/r4w_cfg4_$T.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['validators']; print('   ', round(d['value'], 2), round(d['ms_per_step'], 3))"
  done
done
exit 0
