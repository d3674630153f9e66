#!/bin/bash
# SQ counter pass (one rocprofv3 --pmc run) over a short bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_sq_${TAG:-x}
mkdir -p $OUT
CNT=${COUNTERS:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY}
timeout -s KILL 150 rocprofv3 --pmc $CNT --output-format csv -d $OUT -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu --streams 1 > $OUT/log 2>&1
echo "rc $?"
python3 - <<PY
import csv, collections, glob
f = glob.glob("$OUT/**/run_counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(dict)
for x in csv.DictReader(open(f)):
    n = x['Kernel_Name']
    if 'hbrbc' not in n: continue
    k = n.split('::')[-1].split('(')[0]
    agg[k][x['Counter_Name']] = agg[k].get(x['Counter_Name'], 0) + float(x['Counter_Value'])
for k, v in agg.items():
    print(k, {c: '%.4g' % val for c, val in sorted(v.items())})
PY
