#!/bin/bash
# Round 6, call i: the f4 microbenchmark with the final-exponentiation units
# (timing + SQ_INSTS_VALU), then kernel trace + stats of each instance-mode
# config on the round-6 code (the roofline sources of the line).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
ROOT=$PWD
OUT=gpurun_out/r6i
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 180 ./tools/fp_microbench > $OUT/fp_microbench.jsonl 2>&1
rc=$?; echo "microbench exit $rc"; cat $OUT/fp_microbench.jsonl; if fatal $rc; then exit $rc; fi
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --output-format csv -d $OUT/pmc -o run -- ./tools/fp_microbench > $OUT/pmc.log 2>&1
rc=$?; echo "pmc exit $rc"; if fatal $rc; then exit $rc; fi
export HBRBC_JIT=load
for C in cfg3 cfg5 cfg2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$C -o run -- python3 $ROOT/bench.py --config $C --steps 5 --warmup 1 --no-cpu --mode instances --no-leaf-reuse --f4-checks 0 --no-riders > $OUT/trace_$C.log 2>&1
  rc=$?; echo "trace $C exit $rc"; grep '^{' $OUT/trace_$C.log | tail -1 > $OUT/trace_${C}_bench.json
  if fatal $rc; then exit $rc; fi
done
exit 0
