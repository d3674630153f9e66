#!/bin/bash
# Round 6, call a: GPU parity suite, smoke (with the provenance hash), the
# default bench line (compact, --detail beside it), then the 2-rank gloo
# rehearsal of the multi-GPU line on the new phase order.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r6a
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests exit $rc"; tail -5 $OUT/tests.log
if fatal $rc || [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke exit $rc"; cat $OUT/smoke.log
if fatal $rc; then exit $rc; fi
HBRBC_JIT=load timeout -k 10 500 python bench.py --detail $OUT/detail.json > $OUT/bench.log 2>&1
rc=$?; echo "bench exit $rc"; grep '^{' $OUT/bench.log | tail -1 > $OUT/bench.json; wc -c $OUT/bench.json
if fatal $rc; then exit $rc; fi
HBRBC_JIT=load HBRBC_BENCH_REHEARSE=1 timeout -k 10 500 python bench.py --gpus 2 --steps 3 --warmup 1 --f4-checks 65536 --phase-budget 400 --detail $OUT/detail_g2.json > $OUT/rehearsal_g2.log 2>&1
rc=$?; echo "rehearsal exit $rc"; grep '^{' $OUT/rehearsal_g2.log | tail -1 > $OUT/rehearsal_g2.json; wc -c $OUT/rehearsal_g2.json
exit $rc
