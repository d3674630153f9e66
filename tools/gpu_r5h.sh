#!/bin/bash
# Round 5, call h: state machine with the incremental inbox cursor -- parity
# (every single-root form vs the host restatement) and sm_bench timing.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/r5h
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 600 python -u -m pytest tests/test_rbc_sim.py tests/test_sharded.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests exit $rc"; tail -2 $OUT/tests.log; if fatal $rc; then exit $rc; fi
[ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do
  timeout -k 10 120 python tools/sm_bench.py --reps 7 >> $OUT/sm_bench.jsonl 2>&1
  rc=$?; if fatal $rc; then exit $rc; fi
done
cat $OUT/sm_bench.jsonl
# the Keccak ceiling's own clock: the register-only permutation loop under
# the same GRBM pass as the pipeline's kernels (profiles/r5e_effective_clock.txt)
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $OUT/clk_micro -o run -- ./tools/valu_microbench > $OUT/valu_microbench.txt 2>&1
rc=$?; echo "microbench pmc exit $rc"; if fatal $rc; then exit $rc; fi
grep keccak $OUT/valu_microbench.txt
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/r5h/clk_micro/**/*counter_collection.csv", recursive=True)[0]
rows = {}
for x in csv.DictReader(open(f)):
    key = (x["Dispatch_Id"], x["Kernel_Name"].split("(")[0])
    rows.setdefault(key, {})[x["Counter_Name"]] = float(x["Counter_Value"])
    rows[key]["dur"] = (int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) * 1e-9
for (d, k), v in sorted(rows.items(), key=lambda kv: int(kv[0][0])):
    if "keccak" in k and v["dur"] > 1e-4:
        print("%-30s %8.3f ms clock %.2f GHz" % (k[-30:], v["dur"] * 1e3, v["GRBM_GUI_ACTIVE"] / v["dur"] / 8e9))
PY
exit 0
