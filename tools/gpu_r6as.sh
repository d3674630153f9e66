#!/bin/bash
# Round 6, call as: the headline (cfg3 instance mode) with kernels.hip scheduled
# by other AMDGPU machine-scheduler strategies (hbbft_amd/libhbrbc_k<strategy>.so)
# against the default; alternating, twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp HBRBC_JIT=load
OUT=gpurun_out/r6as_headline_sched_strategy_ab.txt
mkdir -p gpurun_out/r6as
for rep in 1 2; do
  for L in libhbrbc.so libhbrbc_kmax-ilp.so libhbrbc_kiterative-maxocc.so libhbrbc_kiterative-ilp.so; do
    HBRBC_LIB=$PWD/hbbft_amd/$L timeout -k 10 300 python bench.py --mode instances --no-riders --no-cpu --f4-checks 0 --detail gpurun_out/r6as/detail_$L.json > gpurun_out/r6as/bench_$L.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "$L bench exit $rc"; tail -5 gpurun_out/r6as/bench_$L.log; exit $rc; }
    python3 - gpurun_out/r6as/detail_$L.json $L $rep <<'PY' | tee -a $OUT
import json, sys
d = json.load(open(sys.argv[1]))
st = d["stages_ms_per_step"]
print("%s rep %s: %.2f GB/s, ms/step %.2f, leaf_reuse %.1f, encode %.2f leaf_hash %.2f validate %.2f reconstruct %.2f"
      % (sys.argv[2], sys.argv[3], d["value"], d["ms_per_step"], (d.get("leaf_reuse") or {}).get("value", 0),
         st["encode"], st["leaf_hash"], st["validate"], st["reconstruct"]))
PY
  done
done
exit 0
