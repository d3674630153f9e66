#!/bin/bash
# Round 5, call b: calibration with the rows16 pattern, the bench-line test,
# and the driver's default bench command (erase stage, cfg2 / cfg5 riders).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
export PYTHONUNBUFFERED=1 TMPDIR=/tmp HBRBC_JIT=load
OUT=$ROOT/gpurun_out/r5b
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 60 $ROOT/tools/fetch_calib > $OUT/known.json 2> $OUT/known.err
rc=$?; echo "calib exit $rc"; if fatal $rc; then exit $rc; fi
for C in FETCH_SIZE WRITE_SIZE; do
  NAME=$(echo $C | tr 'A-Z' 'a-z')
  timeout -s KILL 60 rocprofv3 --pmc $C --output-format csv -d $OUT/calib_$NAME -o run -- $ROOT/tools/fetch_calib > $OUT/calib_$NAME.log 2>&1
  rc=$?; echo "pmc $NAME exit $rc"; if fatal $rc; then exit $rc; fi
done
python3 tools/fetch_calib.py $OUT/known.json $OUT/calib_fetch_size $OUT/calib_write_size $OUT/fetch_calibration.json > /dev/null
grep -A1 '"fetch_factor"' $OUT/fetch_calibration.json | head -20
timeout -k 10 400 python -u -m pytest tests/test_bench.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/test_bench.log 2>&1
rc=$?; echo "test_bench exit $rc"; tail -3 $OUT/test_bench.log; if fatal $rc; then exit $rc; fi
timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.log 2> $OUT/bench.err
rc=$?; echo "bench exit $rc"; grep '^{' $OUT/bench.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print('head', round(d['value'],2), round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['stages_ms_per_step'].items()})
for k in ('leaf_reuse','validators','validators_cfg4','cfg2','cfg5','threshold_decrypt'):
    v=d.get(k) or {}
    print(k, v.get('error') or (round(v.get('value',0),2), round(v.get('ms_per_step',0),2)))
print('cfg2 em', d['cfg2'].get('encode_merkle',{}).get('value'))
print('cfg5 stages', d['cfg5'].get('stages_ms_per_step'))
"
exit $rc
