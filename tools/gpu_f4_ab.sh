#!/bin/bash
# f4 A/B over library builds (LIBS="libhbrbc.so libhbrbc_x.so ..." under
# hbbft_amd/): pairing parity tests, then the grouped-check microbench under a
# kernel trace (per-kernel average ms) for each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
for L in ${LIBS:-libhbrbc.so}; do
  export HBRBC_LIB=$PWD/hbbft_amd/$L
  timeout -k 10 300 python -u -m pytest tests/test_pairing.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/f4ab_tests_$(basename $L).log 2>&1
  rc=$?; echo "$L tests exit $rc"; [ $rc -ne 0 ] && exit $rc
  OUT=gpurun_out/f4ab_$(basename $L)
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 tools/bench_pairing.py --prepared --n 262144 --reps 3 > $OUT.log 2>&1
  rc=$?; echo "$L bench exit $rc"; [ $rc -ne 0 ] && exit $rc
  tail -1 $OUT.log
  python3 - $OUT <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "miller" in r["Name"] or "final_exp" in r["Name"] or "prepare" in r["Name"]:
            print("   %-40s %8.2f ms" % (r["Name"][:40], float(r["AverageNs"]) / 1e6))
PY
done
exit 0
