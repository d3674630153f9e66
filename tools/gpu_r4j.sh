#!/bin/bash
# Round 4, call j: the overlapped state machine in validator mode (A/B against
# --no-sm-overlap, cfg3 and cfg4 objects), the global-records read forms on
# tools/sm_bench.py, then the full GPU suite, smoke, the default bench line and
# the 2-rank gloo rehearsal (tools/gpu_round.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 600 python -u -m pytest tests/test_sharded.py tests/test_rbc_sim.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4j_gpu_tests.log 2>&1
rc=$?; echo "tests exit $rc"; tail -2 gpurun_out/r4j_gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for i in 1 2; do
  for O in "" "--no-sm-overlap"; do
    for C in cfg3 cfg4; do
      HBRBC_JIT=load timeout -k 10 300 python bench.py --mode validators --config $C --steps 10 --warmup 2 --no-cpu --f4-checks 0 $O > gpurun_out/r4j_v_${C}_${O:-ov}_$i.log 2>&1
      rc=$?; echo "validators $C [$O] $i exit $rc"; if fatal $rc; then exit $rc; fi
      grep '^{' gpurun_out/r4j_v_${C}_${O:-ov}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['validators']; print('   ', round(d['value'], 2), round(d['ms_per_step'], 3), {k: round(v, 3) for k, v in d['stages_ms_per_step'].items() if k.startswith('state') or k in ('leaf_hash', 'validate')})"
    done
  done
done
exit 0
