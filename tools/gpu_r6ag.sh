#!/bin/bash
# Round 6, call ag: f4 with the G2 preparation split into a check wave and a
# line wave per 64 points (HB_G2_SPLIT=1, default libhbrbc.so) against one
# lane doing both (hbbft_amd/libhbrbc_ns.so): pairing tests + kernel times,
# then the bench's f4 leg (side-stream G1 preparation, as in the line), twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/r6ag_f4_g2_split_ab.txt
mkdir -p gpurun_out
LIBS="libhbrbc.so libhbrbc_ns.so" bash tools/gpu_f4_ab.sh 2>&1 | grep -v "^W2026" | tee -a $OUT
rc=${PIPESTATUS[0]}; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for L in libhbrbc.so libhbrbc_ns.so; do
    HBRBC_LIB=$PWD/hbbft_amd/$L timeout -k 10 300 python bench.py --mode instances --count 1024 --no-riders --no-cpu --f4-steps 5 --steps 3 --warmup 1 > gpurun_out/r6ag_bench_$L.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "$L bench exit $rc"; tail -5 gpurun_out/r6ag_bench_$L.log; exit $rc; }
    python3 - gpurun_out/r6ag_bench_$L.log $L $rep <<'PY' | tee -a $OUT
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
t = json.loads(line).get("threshold_decrypt") or {}
print("bench f4 %s rep %s: %s checks/s, ms/step %s" % (sys.argv[2], sys.argv[3], t.get("value"), t.get("ms_per_step")))
PY
  done
done
exit 0
