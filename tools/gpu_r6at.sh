#!/bin/bash
# Round 6, call at: final validation (f4 preparation refactor) -- GPU suite, smoke
# (provenance hash), the default bench line with --detail, and the kernel
# trace + stats of the same default command (profiles/).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
ROOT=$PWD
OUT=gpurun_out/r6at
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests exit $rc"; tail -3 $OUT/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke exit $rc"; cat $OUT/smoke.log; if [ $rc -ne 0 ]; then exit $rc; fi
export HBRBC_JIT=load
timeout -k 10 500 python bench.py --detail $OUT/detail.json > $OUT/bench.log 2>&1
rc=$?; echo "bench exit $rc"; grep '^{' $OUT/bench.log | tail -1 > $OUT/bench.json; wc -c $OUT/bench.json
if fatal $rc; then exit $rc; fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $ROOT/bench.py --no-cpu --detail $OUT/detail_traced.json > $OUT/trace.log 2>&1
rc=$?; echo "trace exit $rc"; grep '^{' $OUT/trace.log | tail -1 > $OUT/bench_traced.json
exit $rc
