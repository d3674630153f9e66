#!/bin/bash
# Round 6, call q: list the gfx950 counters, then an instruction-cache pass
# over the tower microbenchmark (is the 80 KB straight-line cyclotomic
# squaring fetch-bound?).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r6q
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1
rc=$?; echo "list exit $rc"; grep -i -E "SQC_ICACHE|SQC_INST|ICACHE|SQ_IFETCH|SQ_WAIT_INST" $OUT/counters.txt | head -40
if fatal $rc; then exit $rc; fi
C=$(grep -o -E "SQC_ICACHE_(MISSES|HITS|REQ)[A-Z_]*" $OUT/counters.txt | sort -u | head -3 | tr '\n' ' ')
echo "counters: $C"
if [ -n "$C" ]; then
  timeout -s KILL 120 rocprofv3 --pmc $C SQ_INSTS_VALU --output-format csv -d $OUT/pmc -o run -- ./tools/fp_microbench > $OUT/pmc.log 2>&1
  rc=$?; echo "pmc exit $rc"
fi
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU --output-format csv -d $OUT/pmc2 -o run -- ./tools/fp_microbench > $OUT/pmc2.log 2>&1
rc=$?; echo "pmc2 exit $rc"
exit 0
