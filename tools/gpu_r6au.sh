#!/bin/bash
# Round 6, call au: the f4 leg with pairing.hip built under scheduler tuning
# flags (-mllvm -amdgpu-use-amdgpu-trackers=1, ...-disable-unclustered-high-rp-
# reschedule=1, ...-disable-clustered-low-occupancy-reschedule=1) vs the default.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/r6au_f4_sched_strategy_ab.txt
mkdir -p gpurun_out/r6au
for rep in 1 2; do
  for L in libhbrbc.so libhbrbc_trk.so libhbrbc_nohrp.so libhbrbc_noclus.so; do
    HBRBC_LIB=$PWD/hbbft_amd/$L timeout -k 10 300 python bench.py --mode instances --count 1024 --no-riders --no-cpu --f4-steps 5 --steps 3 --warmup 1 > gpurun_out/r6au/bench_$L.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "$L bench exit $rc"; tail -5 gpurun_out/r6au/bench_$L.log; exit $rc; }
    python3 - gpurun_out/r6au/bench_$L.log $L $rep <<'PY' | tee -a $OUT
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
t = json.loads(line).get("threshold_decrypt") or {}
print("bench f4 %s rep %s: %s checks/s, ms/step %s" % (sys.argv[2], sys.argv[3], t.get("value"), t.get("ms_per_step")))
PY
  done
done
exit 0
