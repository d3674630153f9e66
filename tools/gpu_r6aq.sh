#!/bin/bash
# Round 6, call aq: the f4 leg with step i + 1's preparations enqueued beside
# step i's Miller loop (HBRBC_BENCH_F4_SIDE=6) against mode 3, alternating,
# twice; then a kernel trace of mode 6.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/r6aq_f4_prep_streams_ab.txt
mkdir -p gpurun_out/r6aq
for rep in 1 2; do
  for M in 6 3; do
    HBRBC_BENCH_F4_SIDE=$M timeout -k 10 300 python bench.py --mode instances --count 1024 --no-riders --no-cpu --f4-steps 5 --steps 3 --warmup 1 > gpurun_out/r6aq/bench_$M.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "mode $M bench exit $rc"; tail -5 gpurun_out/r6aq/bench_$M.log; exit $rc; }
    python3 - gpurun_out/r6aq/bench_$M.log $M $rep <<'PY' | tee -a $OUT
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
t = json.loads(line).get("threshold_decrypt") or {}
print("f4 side mode %s rep %s: %s checks/s, ms/step %s" % (sys.argv[2], sys.argv[3], t.get("value"), t.get("ms_per_step")))
PY
  done
done
HBRBC_BENCH_F4_SIDE=6 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6aq/trace -o run -- python3 bench.py --mode instances --count 1024 --no-riders --no-cpu --f4-steps 5 --steps 3 --warmup 1 > gpurun_out/r6aq/trace.log 2>&1
rc=$?; echo "trace exit $rc"; exit $rc
