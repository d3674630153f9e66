#!/bin/bash
# Round 6, call an: cfg5 (N=250, 4 MiB x 4096, worst-case decode) with two step
# pipelines on the contexts' own streams (--ipipes 2) against one; twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp HBRBC_JIT=load
OUT=gpurun_out/r6an_cfg5_pipes_ab.txt
mkdir -p gpurun_out/r6an
for rep in 1 2; do
  for P in 2 1; do
    timeout -k 10 300 python bench.py --config cfg5 --mode instances --no-riders --no-cpu --f4-checks 0 --ipipes $P --detail gpurun_out/r6an/detail_$P.json > gpurun_out/r6an/bench_$P.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "pipes $P bench exit $rc"; tail -5 gpurun_out/r6an/bench_$P.log; exit $rc; }
    python3 - gpurun_out/r6an/detail_$P.json $P $rep <<'PY' | tee -a $OUT
import json, sys
d = json.load(open(sys.argv[1]))
print("cfg5 pipes %s rep %s: %.2f GB/s, ms/step %.2f, stages %s" % (sys.argv[2], sys.argv[3], d["value"], d["ms_per_step"], {k: round(v, 2) for k, v in d["stages_ms_per_step"].items()}))
PY
  done
done
exit 0
