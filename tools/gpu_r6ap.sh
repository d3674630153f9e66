#!/bin/bash
# Round 6, call ap: the 2-rank gloo rehearsal of the multi-GPU line on the
# final code (f4 preparation on three streams, split G2 preparation).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 HBRBC_JIT=load
OUT=gpurun_out/r6ap
mkdir -p $OUT
HBRBC_BENCH_REHEARSE=1 timeout -k 10 900 python bench.py --gpus 2 --steps 3 --warmup 1 --f4-checks 65536 --phase-budget 400 --detail $OUT/detail_g2.json > $OUT/rehearsal_g2.log 2>&1
rc=$?; echo "rehearsal g2 exit $rc"; grep '^{' $OUT/rehearsal_g2.log | tail -1 > $OUT/rehearsal_g2.json; wc -c $OUT/rehearsal_g2.json
exit $rc
