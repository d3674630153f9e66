#!/bin/bash
# Round 5, call s: state-machine sender loop variants (default lib) vs the
# previous build (ab/libhbrbc_base.so).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
export PYTHONUNBUFFERED=1 TMPDIR=/tmp HBRBC_JIT_DIR=$ROOT/hbbft_amd/jit
OUT=gpurun_out/r5s
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 300 python -u -m pytest tests/test_rbc_sim.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests exit $rc"; tail -2 $OUT/tests.log; if fatal $rc; then exit $rc; fi
[ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do
  for L in libhbrbc.so ab/libhbrbc_base.so; do
    HBRBC_LIB=$ROOT/hbbft_amd/$L timeout -k 10 120 python tools/sm_bench.py --reps 7 >> $OUT/sm_bench.jsonl 2>/dev/null
    rc=$?; if fatal $rc; then exit $rc; fi
  done
done
python3 -c "
import json
for l in open('$OUT/sm_bench.jsonl'):
    d = json.loads(l); print(d['lib'], d['n'], round(d['ms_median'], 3), round(d['ms_min'], 3))
"
exit 0
