#!/bin/bash
# Round 6, call t: the tower microbenchmark with the three Fp products of an
# Fp2 product serialised (HB_FP2_SERIAL=1, tools/fp_microbench_serial) against
# the default build, twice each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r6t
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
for rep in 1 2; do
for B in fp_microbench fp_microbench_serial; do
  timeout -k 10 180 ./tools/$B > $OUT/${B}_${rep}.jsonl 2>&1
  rc=$?; echo "$B exit $rc"; if fatal $rc; then exit $rc; fi
done
done
python3 - <<'PY'
import json
for rep in (1, 2):
    a = {d["kernel"]: d["ms"] for d in map(json.loads, open("gpurun_out/r6t/fp_microbench_%d.jsonl" % rep)) }
    b = {d["kernel"]: d["ms"] for d in map(json.loads, open("gpurun_out/r6t/fp_microbench_serial_%d.jsonl" % rep)) }
    for k in a:
        print("rep %d %-12s default %8.3f ms  serial %8.3f ms  %.3f" % (rep, k, a[k], b[k], b[k] / a[k]))
PY
exit 0
