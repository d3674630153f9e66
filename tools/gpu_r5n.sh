#!/bin/bash
# Round 5, call n: f4 -- the cyclotomic square inlined into exp_by_x's loop
# (hbbft_amd/ab/libhbrbc_cyc.so, -DHB_INL_CYC=1; _cycw1: also 1 wave/SIMD),
# pairing parity on each variant, then grouped checks timed alternately.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
export PYTHONUNBUFFERED=1 TMPDIR=/tmp HBRBC_JIT_DIR=$ROOT/hbbft_amd/jit
OUT=gpurun_out/r5n
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
for L in ab/libhbrbc_cyc.so ab/libhbrbc_cycw1.so; do
  T=$(basename $L .so)
  HBRBC_LIB=$ROOT/hbbft_amd/$L timeout -k 10 300 python -u -m pytest tests/test_pairing.py -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/tests_$T.log 2>&1
  rc=$?; echo "$T tests exit $rc"; tail -1 $OUT/tests_$T.log; if fatal $rc; then exit $rc; fi
  [ $rc -ne 0 ] && exit $rc
done
for rep in 1 2; do
  for L in libhbrbc.so ab/libhbrbc_cyc.so ab/libhbrbc_cycw1.so; do
    HBRBC_LIB=$ROOT/hbbft_amd/$L timeout -k 10 300 python tools/bench_pairing.py --prepared --n 262144 --reps 3 > $OUT/b.log 2>&1
    rc=$?; if fatal $rc; then echo "bench $L exit $rc"; exit $rc; fi
    echo "$L $(grep '^{' $OUT/b.log)" | tee -a $OUT/ab.txt | cut -c1-400
  done
done
exit 0
