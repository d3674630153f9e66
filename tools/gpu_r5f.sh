#!/bin/bash
# Round 5, call f: parity of the coefficient-switch GF kernel, its A/B in the
# cfg3 / cfg4 instance step, then the r5e measurements (state-machine
# profile, effective clock, MFMA encoder study).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
export PYTHONUNBUFFERED=1 TMPDIR=/tmp HBRBC_JIT=load
OUT=$ROOT/gpurun_out/r5f
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
HBRBC_JIT= timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_unframe_fused.py -m gpu -x -q -k "variants or fused" --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests exit $rc"; tail -3 $OUT/tests.log; if fatal $rc; then exit $rc; fi
[ $rc -ne 0 ] && exit $rc
for CFG in cfg3 cfg4; do
  for GF in ${GF_LIST:-bitslice switch bitslice switch}; do
    HBRBC_GF=$GF timeout -k 10 300 python bench.py --config $CFG --mode instances --steps 6 --warmup 2 --no-cpu --f4-checks 0 --no-leaf-reuse > $OUT/ab_${CFG}_$GF.log 2>&1
    rc=$?; if fatal $rc; then echo "bench $CFG $GF exit $rc"; exit $rc; fi
    grep '^{' $OUT/ab_${CFG}_$GF.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); s=d['stages_ms_per_step']; print('$CFG $GF', round(d['value'],2), 'GB/s  reconstruct', round(s['reconstruct'],3), 'ms  encode', round(s['encode'],3))" | tee -a $OUT/ab.txt
  done
done
[ -z "$NO_R5E" ] && bash tools/gpu_r5e.sh
exit 0
