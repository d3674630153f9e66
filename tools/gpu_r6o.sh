#!/bin/bash
# Round 6, call o: prepared G1 keys -- pairing parity tests, the f4 profile
# (trace + SQ counters -> VALU ops per check), the default line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/r6o
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 600 python -u -m pytest tests/test_pairing.py tests/test_bench.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests exit $rc"; tail -3 $OUT/tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_f4_prof.sh > $OUT/f4_prof.log 2>&1
rc=$?; echo "f4 prof exit $rc"; tail -40 $OUT/f4_prof.log | grep -A40 '^{' > $OUT/pairing_valu_ops.json; if fatal $rc; then exit $rc; fi
export HBRBC_JIT=load
timeout -k 10 500 python bench.py --detail $OUT/detail.json > $OUT/bench.log 2>&1
rc=$?; echo "bench exit $rc"; grep '^{' $OUT/bench.log | tail -1 > $OUT/bench.json; wc -c $OUT/bench.json
exit $rc
