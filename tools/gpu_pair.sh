#!/bin/bash
# f4 pairing microbench: plain checks (multi-Miller) and prepared grouped
# checks, then optionally a rocprofv3 kernel trace of the prepared form.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
N=${N:-16384}
timeout -k 10 300 python tools/bench_pairing.py --n $N --reps 3 || exit $?
timeout -k 10 300 python tools/bench_pairing.py --n $N --reps 3 --prepared || exit $?
if [ -n "$PROF" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_pair -o run -- python3 tools/bench_pairing.py --n $N --reps 2 --prepared > gpurun_out/prof_pair.log 2>&1
  rc=$?; echo "prof exit $rc"; find gpurun_out/prof_pair -name "*kernel_stats.csv" -exec cat {} \;
fi
