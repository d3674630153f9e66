#!/bin/bash
# Round 5, call a: FETCH_SIZE / WRITE_SIZE calibration on known byte counts in
# the kernels' own access patterns (tools/fetch_calib.hip), and a kernel trace
# of the 2-stream instance bench to read which hardware queue each stream used.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
export PYTHONUNBUFFERED=1 TMPDIR=/tmp HBRBC_JIT=load
OUT=$ROOT/gpurun_out/r5a
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/calib_trace -o run -- $ROOT/tools/fetch_calib > $OUT/known.json 2> $OUT/calib_trace.err
rc=$?; echo "calib trace exit $rc"; cat $OUT/known.json
if fatal $rc; then exit $rc; fi
for C in FETCH_SIZE WRITE_SIZE; do
  NAME=$(echo $C | tr 'A-Z' 'a-z')
  timeout -s KILL 60 rocprofv3 --pmc $C --output-format csv -d $OUT/calib_$NAME -o run -- $ROOT/tools/fetch_calib > $OUT/calib_$NAME.log 2>&1
  rc=$?; echo "pmc $NAME exit $rc"
  if fatal $rc; then exit $rc; fi
done
python3 tools/fetch_calib.py $OUT/known.json $OUT/calib_fetch_size $OUT/calib_write_size $OUT/fetch_calibration.json
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/streams2 -o run -- python3 $ROOT/bench.py --mode instances --streams 2 --steps 3 --warmup 1 --no-cpu --f4-checks 0 --no-leaf-reuse > $OUT/streams2.log 2>&1
rc=$?; echo "streams2 exit $rc"; grep '^{' $OUT/streams2.log | head -c 400; echo
if fatal $rc; then exit $rc; fi
python3 tools/queue_map.py $(find $OUT/streams2 -name "*kernel_trace.csv") hbrbc > $OUT/queue_map.json
python3 tools/queue_map.py $(find $OUT/streams2 -name "*kernel_trace.csv") > $OUT/queue_map_all.json
cat $OUT/queue_map.json
exit 0
