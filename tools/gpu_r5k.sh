#!/bin/bash
# Round 5, call k: the committed profile set at the round-5 default for the
# headline (cfg3) and the two riders (cfg2, cfg5): kernel trace + stats, and
# FETCH_SIZE / WRITE_SIZE / SQ_INSTS_VALU passes (tools/profile.sh), so
# roofline.profiled, roofline.traffic and the VALU-per-permutation figure of
# every object of the line come from this round's code.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp HBRBC_JIT=load
for C in cfg3 cfg2 cfg5; do
  TAG=r5k_$C BENCH_ARGS="--config $C --steps 5 --warmup 1 --no-cpu --mode instances --no-leaf-reuse --f4-checks 0 --no-riders" \
  PMC_ARGS="--config $C --steps 1 --warmup 1 --no-cpu --mode instances --no-verify --no-leaf-reuse --f4-checks 0 --no-riders" bash tools/profile.sh
  rc=$?; echo "profile $C exit $rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
