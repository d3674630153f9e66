#!/bin/bash
# Round 6, call c: cfg2 with two step pipelines on the contexts' own streams
# -- kernel trace + queue map (do the pipes overlap?), then the A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp HBRBC_JIT=load
ROOT=$PWD
OUT=gpurun_out/r6c
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python3 $ROOT/bench.py --config cfg2 --mode instances --ipipes 2 --steps 4 --warmup 2 --no-cpu --f4-checks 0 > $OUT/trace.log 2>&1
rc=$?; echo "trace exit $rc"; if fatal $rc; then exit $rc; fi
python3 tools/queue_map.py $(find $OUT/trace -name "*kernel_trace.csv") hbrbc > $OUT/queue_map.json
cat $OUT/queue_map.json | head -40
summ() { grep '^{' $1 | tail -1 | python3 -c "
import json,sys; d=json.load(sys.stdin)
print('$2', 'value', d['value'], 'ms', d['ms_per_step'], 'em', d.get('encode_merkle'), 'stages', {k: round(v,2) for k,v in d['stages_ms_per_step'].items()})" | tee -a $OUT/summary.txt; }
for rep in 1 2; do
for P in 1 2 3; do
  timeout -k 10 300 python bench.py --config cfg2 --mode instances --ipipes $P --no-cpu --f4-checks 0 > $OUT/cfg2_p${P}_${rep}.log 2>&1
  rc=$?; if fatal $rc; then exit $rc; fi
  summ $OUT/cfg2_p${P}_${rep}.log "cfg2 pipes=$P rep=$rep"
done
done
exit 0
