#!/bin/bash
# Round 4, call p: step pipelines side by side in validator mode (--vpipes 2:
# two ShardedBroadcast objects on their own streams, step i on pipe i % 2)
# against one pipeline, cfg3 and cfg4; their test.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 300 python -u -m pytest tests/test_sharded.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r4p_tests.log 2>&1
rc=$?; echo "tests exit $rc"; tail -2 gpurun_out/r4p_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
export HBRBC_JIT=load
for i in 1 2; do
  for C in cfg3 cfg4; do
    for P in 1 2; do
      timeout -k 10 300 python bench.py --mode validators --config $C --steps 12 --warmup 2 --no-cpu --f4-checks 0 --vpipes $P > gpurun_out/r4p_${C}_p${P}_$i.log 2>&1
      rc=$?; echo "$C vpipes $P run $i exit $rc"; if fatal $rc; then exit $rc; fi
      grep '^{' gpurun_out/r4p_${C}_p${P}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['validators']; print('   ', round(d['value'], 2), round(d['ms_per_step'], 3))"
    done
  done
done
exit 0
