#!/bin/bash
# Round 6, call ab: f4 profile on the final default (serialised Fp2, f^|x| one unit) (VALU ops per
# check for the roofline), then the default line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/r6ab
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
bash tools/gpu_f4_prof.sh > $OUT/f4_prof.log 2>&1
rc=$?; echo "f4 prof exit $rc"; if fatal $rc || [ $rc -ne 0 ]; then exit $rc; fi
export HBRBC_JIT=load
timeout -k 10 500 python bench.py --detail $OUT/detail.json > $OUT/bench.log 2>&1
rc=$?; echo "bench exit $rc"; grep '^{' $OUT/bench.log | tail -1 > $OUT/bench.json; wc -c $OUT/bench.json
exit $rc
