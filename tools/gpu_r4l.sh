#!/bin/bash
# Round 4, call l: kernel trace of the validator mode (cfg3 + cfg4, state
# machine not overlapped so every kernel runs alone), and the decode list's
# pair-lane cut-off A/B (HBRBC_LIST_PAIR_BELOW=0: one lane per sponge).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp HBRBC_JIT=load
mkdir -p gpurun_out
ARGS="--mode validators --steps 4 --warmup 1 --no-cpu --f4-checks 0 --no-sm-overlap"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r4l_v -o run -- python3 bench.py $ARGS > gpurun_out/r4l_trace.log 2>&1
rc=$?; echo "trace exit $rc"; [ $rc -ne 0 ] && exit $rc
python3 - <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/prof_r4l_v/**/*kernel_stats.csv", recursive=True):
    for r in list(csv.DictReader(open(f)))[:16]:
        print("  %-64s %5s %9.1f us" % (r["Name"][:64], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
for B in 0 262144; do
  HBRBC_LIST_PAIR_BELOW=$B timeout -k 10 300 python bench.py $ARGS > gpurun_out/r4l_pair$B.log 2>&1
  rc=$?; echo "pair-below $B exit $rc"; [ $rc -ne 0 ] && exit $rc
  grep '^{' gpurun_out/r4l_pair$B.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
for k in ('validators', 'validators_cfg4'):
    v = d.get(k)
    if v: print('   ', k, round(v['value'], 2), round(v['ms_per_step'], 3), {a: round(b, 3) for a, b in v['stages_ms_per_step'].items()})"
done
exit 0
