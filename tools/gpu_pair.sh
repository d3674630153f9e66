#!/bin/bash
# f4 pairing microbench: occupancy variants, then a rocprofv3 kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
N=${N:-16384}
for w in ${WAVES:-1 2 4}; do
  HBRBC_PAIR_WAVES=$w timeout -k 10 300 python tools/bench_pairing.py --n $N --reps 3 || exit $?
done
if [ -n "$PROF" ]; then
  HBRBC_PAIR_WAVES=$PROF timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_pair -o run -- python3 tools/bench_pairing.py --n $N --reps 2 > gpurun_out/prof_pair.log 2>&1
  rc=$?; echo "prof exit $rc"; find gpurun_out/prof_pair -name "*kernel_stats.csv" -exec cat {} \;
fi
