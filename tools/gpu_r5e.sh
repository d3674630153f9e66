#!/bin/bash
# Round 5, call e: (1) state machine at N=64 / N=128 alone -- kernel trace per
# round and one SQ counter pass; (2) effective clock of every kernel of the
# cfg3 instance step (GRBM_GUI_ACTIVE cycles / dispatch duration).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
export PYTHONUNBUFFERED=1 TMPDIR=/tmp HBRBC_JIT=load
OUT=$ROOT/gpurun_out/r5e
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
HBRBC_JIT= timeout -k 10 600 python -u -m pytest tests/test_rbc_sim.py tests/test_layouts.py tests/test_drop_rows.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests exit $rc"; tail -2 $OUT/tests.log; if fatal $rc; then exit $rc; fi
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/sm_trace -o run -- python3 $ROOT/tools/sm_bench.py --reps 3 > $OUT/sm_trace.log 2>&1
rc=$?; echo "sm trace exit $rc"; grep '^{' $OUT/sm_trace.log; if fatal $rc; then exit $rc; fi
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAVES SQ_INSTS_BRANCH --output-format csv -d $OUT/sm_pmc -o run -- python3 $ROOT/tools/sm_bench.py --reps 1 > $OUT/sm_pmc.log 2>&1
rc=$?; echo "sm pmc exit $rc"; if fatal $rc; then exit $rc; fi
timeout -s KILL 180 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $OUT/clk -o run -- python3 $ROOT/bench.py --steps 2 --warmup 1 --no-cpu --mode instances --no-leaf-reuse --f4-checks 0 --no-verify > $OUT/clk.log 2>&1
rc=$?; echo "clock pmc exit $rc"; if fatal $rc; then exit $rc; fi
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/r5e/clk/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: [0.0, 0.0, 0])
rows = {}
for x in csv.DictReader(open(f)):
    key = (x["Dispatch_Id"], x["Kernel_Name"].split("(")[0][-60:])
    rows.setdefault(key, {})[x["Counter_Name"]] = float(x["Counter_Value"])
    rows[key]["dur"] = (int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) * 1e-9
for (d, k), v in rows.items():
    if "GRBM_GUI_ACTIVE" in v and v["dur"] > 1e-4:
        a = acc[k]; a[0] += v["GRBM_GUI_ACTIVE"]; a[1] += v["dur"]; a[2] += 1
for k, (c, t, n) in sorted(acc.items(), key=lambda kv: -kv[1][1]):
    print("%-60s %3d launches %8.2f ms  GUI_ACTIVE/dur = %.3f GHz" % (k, n, t * 1e3 / n, c / t / 1e9))
PY
# (3) the cfg3 FP4-MFMA encoder prototype (tools/mfma_enc.hip): bit-exactness
# against the XOR-network encoder, times alone and beside a leaf-hash launch,
# and its instruction counts
timeout -k 10 120 ./tools/mfma_enc 32768 5 > $OUT/mfma_enc.log 2>&1
rc=$?; echo "mfma_enc exit $rc"; cat $OUT/mfma_enc.log; if fatal $rc; then exit $rc; fi
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d $OUT/mfma_pmc -o run -- ./tools/mfma_enc 32768 1 > $OUT/mfma_pmc.log 2>&1
rc=$?; echo "mfma pmc exit $rc"; if fatal $rc; then exit $rc; fi
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/r5e/mfma_pmc/**/*counter_collection.csv", recursive=True)[0]
tot = collections.defaultdict(lambda: collections.defaultdict(float)); ids = collections.defaultdict(set)
for x in csv.DictReader(open(f)):
    k = x["Kernel_Name"].split("(")[0][-50:]
    tot[k][x["Counter_Name"]] += float(x["Counter_Value"]); ids[k].add(x["Dispatch_Id"])
for k, v in tot.items():
    n = len(ids[k])
    print(k, n, {c: round(val / n) for c, val in v.items()})
PY
exit 0
