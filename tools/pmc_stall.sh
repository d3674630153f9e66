#!/bin/bash
# Stall/issue counters of the GF kernels (specialised encoders, generic
# reconstruct) over one bench step: one rocprofv3 --pmc run per counter group
# (never combined with traces), then a per-kernel summary.
#   TAG=enc CONFIG=cfg3 bash tools/pmc_stall.sh     -> gpurun_out/pmc_<tag>/summary.txt
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
export TMPDIR=/tmp
OUT=$ROOT/gpurun_out/pmc_${TAG:-stall}
mkdir -p $OUT
REGEX=${REGEX:-hbrbc_enc|hbrbc_dec|gf_bitslice|leaf_hash|validate_kernel}
ARGS="--config ${CONFIG:-cfg3} --steps 1 --warmup 1 --no-cpu --mode ${MODE:-instances} --no-verify --no-leaf-reuse --f4-checks 0"
i=0
# SETS="group1|group2|..." replaces the default counter groups
if [ -n "$SETS" ]; then IFS='|' read -r -a GROUPS_ <<< "$SETS"; else GROUPS_=(); fi
if [ ${#GROUPS_[@]} -gt 0 ]; then set -- "${GROUPS_[@]}"; else set -- "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM" \
         "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD" \
         "FETCH_SIZE" "WRITE_SIZE"; fi
for C in "$@"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $C --kernel-include-regex "$REGEX" --output-format csv -d $OUT/p$i -o run -- python3 $ROOT/bench.py $ARGS > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i exit $rc"
  case $rc in 0) ;; *) tail -5 $OUT/p$i.log; exit $rc;; esac
done
python3 - "$OUT" > $OUT/summary.txt <<'EOF'
import collections, csv, glob, re, sys
out = sys.argv[1]
tot = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in glob.glob(out + "/p*/**/run_counter_collection.csv", recursive=True):
    for x in csv.DictReader(open(f)):
        m = re.search(r"(hbrbc_(enc|dec)_\w+|\w+_kernel(<[^>]*>)?)", x["Kernel_Name"])
        k = m.group(1) if m else x["Kernel_Name"][:50]
        tot[k][x["Counter_Name"]] += float(x["Counter_Value"])
        disp[(k, x["Counter_Name"])].add(x["Dispatch_Id"])
for k in sorted(tot):
    print(k)
    for c in sorted(tot[k]):
        print("   %-26s %16.0f" % (c, tot[k][c] / max(1, len(disp[(k, c)]))))
EOF
cat $OUT/summary.txt
