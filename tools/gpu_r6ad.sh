#!/bin/bash
# Round 6, call ad: shares decoded beside the G2 preparation
# (hbrbc_pairing_check_prepared_pts) -- pairing tests, the f4 leg in its three
# modes (HBRBC_BENCH_F4_SIDE 0 / 1 / 2), then the f4 profile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp HBRBC_JIT=load
OUT=gpurun_out/r6ad
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 600 python -u -m pytest tests/test_pairing.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests exit $rc"; tail -2 $OUT/tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
for rep in 1 2; do
for S in 1 2; do
  HBRBC_BENCH_F4_SIDE=$S timeout -k 10 300 python bench.py --mode instances --no-riders --no-leaf-reuse --no-cpu --count 1024 --steps 2 --f4-steps 6 > $OUT/f4_s${S}_${rep}.log 2>&1
  rc=$?; if fatal $rc; then exit $rc; fi
  grep '^{' $OUT/f4_s${S}_${rep}.log | tail -1 | python3 -c "
import json,sys; d=json.load(sys.stdin); t=d['threshold_decrypt']
print('side=$S rep=$rep', t.get('value'), t.get('ms_per_step'), t.get('error'))" | tee -a $OUT/summary.txt
done
done
bash tools/gpu_f4_prof.sh > $OUT/f4_prof.log 2>&1
rc=$?; echo "f4 prof exit $rc"
exit $rc
