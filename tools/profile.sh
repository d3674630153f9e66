#!/bin/bash
# rocprofv3 passes over one bench configuration: kernel trace + stats, then one
# counter pass per group (FETCH_SIZE, WRITE_SIZE, SQ VALU), each its own run
# as MI355X_MICROARCH.md prescribes.  Output under gpurun_out/prof_<tag>.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
export TMPDIR=/tmp
TAG=${TAG:-r2}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p $OUT
ARGS=${BENCH_ARGS:---steps 5 --warmup 1 --no-cpu --mode instances}
PARGS=${PMC_ARGS:---steps 1 --warmup 1 --no-cpu --mode instances --no-verify --no-leaf-reuse}
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $ROOT/bench.py $ARGS > $OUT/trace.log 2>&1
rc=$?; echo "trace exit $rc"; tail -c 1500 $OUT/trace.log; echo
if fatal $rc; then exit $rc; fi
for C in FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU SQ_WAVES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES"; do
  NAME=$(echo $C | cut -d' ' -f1 | tr 'A-Z' 'a-z')
  timeout -s KILL 180 rocprofv3 --pmc $C --output-format csv -d $OUT/pmc_$NAME -o run -- python3 $ROOT/bench.py $PARGS > $OUT/pmc_$NAME.log 2>&1
  rc=$?; echo "pmc $NAME exit $rc"
  if fatal $rc; then exit $rc; fi
done
find $OUT -name "*stats.csv" | head
