#!/bin/bash
# State machine (f2) check: its GPU tests, then the validator-sharded bench
# objects (cfg3 N=64 and cfg4 N=128) with the state machine's time per step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
TAG=${TAG:-sm}
timeout -k 10 400 python -u -m pytest tests/test_rbc_sim.py tests/test_sharded.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests exit $rc"; tail -3 gpurun_out/${TAG}_tests.log
[ $rc -ne 0 ] && exit $rc
for st in 1 0; do
HBRBC_SM_STAGED=$st HBRBC_JIT=load timeout -k 10 300 python bench.py --mode both --steps 5 --warmup 1 --f4-checks 0 --no-cpu > gpurun_out/${TAG}_bench_st$st.log 2>&1
rc=$?; echo "bench staged=$st exit $rc"
[ $rc -ne 0 ] && exit $rc
python - gpurun_out/${TAG}_bench_st$st.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print("instances", round(d["value"], 2), "GB/s")
for k in ("validators", "validators_cfg4"):
    v = d.get(k)
    if v: print(k, round(v["value"], 2), "GB/s", round(v["ms_per_step"], 3), "ms/step", {a: round(b, 3) for a, b in v["stages_ms_per_step"].items()})
PY
done
exit $rc
