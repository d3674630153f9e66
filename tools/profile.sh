#!/bin/bash
# rocprofv3 passes over the default bench (kernel trace + stats, then one
# counter pass per TCC counter group).  Output under gpurun_out/prof_<tag>.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
cd /tmp 2>/dev/null; export TMPDIR=/tmp; cd - >/dev/null
TAG=${TAG:-r1}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
ARGS=${BENCH_ARGS:---steps 5 --warmup 1 --no-cpu}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.log 2>&1
rc=$?; echo "trace exit $rc"; tail -2 $OUT/trace.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu > $OUT/pmc_fetch.log 2>&1
rc=$?; echo "pmc fetch exit $rc"
case $rc in 124|134|137|139) exit $rc;; esac
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu > $OUT/pmc_write.log 2>&1
rc=$?; echo "pmc write exit $rc"
find $OUT -name "*.csv" | head -20
