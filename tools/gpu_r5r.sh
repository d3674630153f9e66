#!/bin/bash
# Round 5, call r: the lean state-machine kernels -- w4 vs the default-budget
# form at N=128, a kernel trace per round, and the SQ counters per round
# (the r5e set) for the lean kernels.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
export PYTHONUNBUFFERED=1 TMPDIR=/tmp HBRBC_JIT_DIR=$ROOT/hbbft_amd/jit
OUT=gpurun_out/r5r
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 300 python -u -m pytest tests/test_rbc_sim.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests exit $rc"; tail -2 $OUT/tests.log; if fatal $rc; then exit $rc; fi
[ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for W in auto 0 1; do
    if [ $W = auto ]; then unset HBRBC_SM_W4; else export HBRBC_SM_W4=$W; fi
    timeout -k 10 120 python tools/sm_bench.py --reps 7 >> $OUT/sm_bench.jsonl 2>/dev/null
    rc=$?; if fatal $rc; then exit $rc; fi
  done
done
unset HBRBC_SM_W4
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/trace -o run -- python3 $ROOT/tools/sm_bench.py --reps 3 > $ROOT/$OUT/trace.log 2>&1
rc=$?; echo "trace exit $rc"; if fatal $rc; then exit $rc; fi
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAVES SQ_INSTS_BRANCH --output-format csv -d $ROOT/$OUT/pmc -o run -- python3 $ROOT/tools/sm_bench.py --reps 1 > $ROOT/$OUT/pmc.log 2>&1
rc=$?; echo "pmc exit $rc"; if fatal $rc; then exit $rc; fi
cd $ROOT
python3 -c "
import json
for l in open('$OUT/sm_bench.jsonl'):
    d = json.loads(l); print('w4', d['w4'], d['n'], round(d['ms_median'], 3), round(d['ms_min'], 3))
"
exit 0
