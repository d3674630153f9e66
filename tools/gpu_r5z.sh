#!/bin/bash
# Round 5, call z: the LDS-staged encoder reading the next input's planes one
# input ahead (HBRBC_JIT_LDS_PF=1, code object *_Lp_*) -- bit-exactness of the
# cfg3 encoder, then the instance-mode cfg3 line alternating with the default.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r5z
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
HBRBC_JIT_LDS_PF=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "(specialised_encoder_vs_oracle and 22) or (frame_encode_fused and 64) or (pipeline_vs_oracle and 64)" > $OUT/tests.log 2>&1
rc=$?; echo "tests exit $rc"; tail -2 $OUT/tests.log; if fatal $rc; then exit $rc; fi
[ $rc -ne 0 ] && exit $rc
export HBRBC_JIT=load
for rep in 1 2 3; do
  for PF in 0 1; do
    HBRBC_JIT_LDS_PF=$PF timeout -k 10 300 python bench.py --mode instances --steps 6 --warmup 2 --no-cpu --no-riders --f4-checks 0 > $OUT/b_${PF}_${rep}.log 2>&1
    rc=$?; if fatal $rc; then exit $rc; fi
    grep '^{' $OUT/b_${PF}_${rep}.log | tail -1 | python3 -c "
import json,sys; d=json.load(sys.stdin); s=d['stages_ms_per_step']
print('pf $PF', round(d['value'],2), 'encode', round(s['encode'],3), 'reconstruct', round(s['reconstruct'],3))" | tee -a $OUT/summary.txt
  done
done
exit 0
