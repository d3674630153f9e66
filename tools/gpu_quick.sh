#!/bin/bash
# Development round trip: GPU tests, then short instance-mode benches of the
# configs in $CONFIGS (default cfg3 cfg5); stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/gpu_tests.log 2>&1
  rc=$?; echo "tests exit $rc"; tail -4 gpurun_out/gpu_tests.log
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
for c in ${CONFIGS:-cfg3 cfg5}; do
  timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 1 --no-cpu --mode ${MODE:-instances} ${BENCH_EXTRA} > gpurun_out/bench_$c.log 2>&1
  rc=$?; echo "bench $c exit $rc"
  python3 -c "
import json,sys
l=[x for x in open('gpurun_out/bench_$c.log') if x.startswith('{')]
if not l: print(open('gpurun_out/bench_$c.log').read()[-2000:]); sys.exit()
d=json.loads(l[-1]); print('value %.2f GB/s  ms/step %.2f' % (d['value'], d['ms_per_step']))
print({k: round(v,3) for k,v in d['stages_ms_per_step'].items()})
if 'validators' in d: v=d['validators']; print('validators %.2f GB/s ms/step %.2f exch %s' % (v['value'], v['ms_per_step'], v['exchange']))
"
  if fatal $rc || [ $rc -ne 0 ]; then exit $rc; fi
done
