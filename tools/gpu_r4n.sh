#!/bin/bash
# Round 4, call n: (1) the generic reconstruct with input pairs per step
# (HBRBC_GF=bitslice_x2; scalar bit masks, one-sided branches) against the
# one-input form; (2) the balanced rebuilt-row list (one block per CU, one-lane
# rounds + a pair-lane remainder) against all-pair-lane (HBRBC_LIST_FORM=pair),
# validator mode, plus its kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_unframe_fused.py tests/test_sharded.py tests/test_layouts.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r4n_tests.log 2>&1
rc=$?; echo "tests exit $rc"; tail -3 gpurun_out/r4n_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
export HBRBC_JIT=load
for i in 1 2; do
  for G in bitslice bitslice_x2; do
    HBRBC_GF=$G timeout -k 10 300 python bench.py --mode instances --steps 8 --warmup 2 --no-cpu --f4-checks 0 --no-leaf-reuse > gpurun_out/r4n_ab_${G}_$i.log 2>&1
    rc=$?; echo "ab $G $i exit $rc"; if fatal $rc; then exit $rc; fi
    grep '^{' gpurun_out/r4n_ab_${G}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('   ', round(d['value'], 2), round(d['stages_ms_per_step']['reconstruct'], 3))"
  done
  for F in pair mix; do
    HBRBC_LIST_FORM=$F timeout -k 10 300 python bench.py --mode validators --steps 8 --warmup 2 --no-cpu --f4-checks 0 --no-sm-overlap > gpurun_out/r4n_list_${F}_$i.log 2>&1
    rc=$?; echo "list $F $i exit $rc"; if fatal $rc; then exit $rc; fi
    grep '^{' gpurun_out/r4n_list_${F}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['validators']; print('   ', round(d['value'], 2), round(d['stages_ms_per_step']['leaf_hash'], 3))"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r4n_v -o run -- python3 bench.py --mode validators --steps 4 --warmup 1 --no-cpu --f4-checks 0 --no-sm-overlap > gpurun_out/r4n_trace.log 2>&1
rc=$?; echo "trace exit $rc"; if fatal $rc; then exit $rc; fi
python3 - <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/prof_r4n_v/**/*kernel_stats.csv", recursive=True):
    for r in list(csv.DictReader(open(f)))[:6]:
        print("  %-64s %5s %9.1f us" % (r["Name"][:64], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
HBRBC_GF=bitslice_x2 TAG=r4n_gf_x2 CONFIG=cfg3 REGEX="gf_bitslice" \
SETS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA|SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_IFETCH SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE" \
  bash tools/pmc_stall.sh > /dev/null
rc=$?; echo "pmc exit $rc"; cat gpurun_out/pmc_r4n_gf_x2/summary.txt
exit $rc
