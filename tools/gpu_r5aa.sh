#!/bin/bash
# Round 5, call aa: the generic GF kernel with two 32-position groups per lane
# (HBRBC_GF=bitslice_w2: half the coefficient-bit tests per byte) -- the
# variant parity tests (and the fused unframe under it), then the cfg3
# instance-mode line: default vs w2 at 7 / 5 / 4-row passes, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r5aa
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "gf_kernel_variants" > $OUT/tests.log 2>&1
rc=$?; echo "tests exit $rc"; tail -2 $OUT/tests.log; if fatal $rc; then exit $rc; fi
[ $rc -ne 0 ] && exit $rc
HBRBC_GF=bitslice_w2 timeout -k 10 400 python -u -m pytest tests/test_unframe_fused.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests_uf.log 2>&1
rc=$?; echo "unframe tests (w2) exit $rc"; tail -2 $OUT/tests_uf.log; if fatal $rc; then exit $rc; fi
[ $rc -ne 0 ] && exit $rc
export HBRBC_JIT=load
for rep in 1 2; do
  for V in "bitslice 7" "bitslice_w2 7" "bitslice_w2 5" "bitslice_w2 4"; do
    set -- $V
    HBRBC_GF=$1 HBRBC_RT_REC=$2 timeout -k 10 300 python bench.py --mode instances --steps 6 --warmup 2 --no-cpu --no-riders --f4-checks 0 > $OUT/b_$1_$2_$rep.log 2>&1
    rc=$?; if fatal $rc; then exit $rc; fi
    grep '^{' $OUT/b_$1_$2_$rep.log | tail -1 | python3 -c "
import json,sys; d=json.load(sys.stdin); s=d['stages_ms_per_step']
print('$1 rt $2', round(d['value'],2), 'reconstruct', round(s['reconstruct'],3), 'encode', round(s['encode'],3))" | tee -a $OUT/summary.txt
  done
done
exit 0
