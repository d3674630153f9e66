#!/bin/bash
# MFMA GF(2) prototype: exactness + issue-bound timing, and its rocprof kernel stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/mfma
timeout -k 10 120 ./tools/mfma_gf 1024 > gpurun_out/mfma/run.log 2>&1
rc=$?; echo "mfma exit $rc"; cat gpurun_out/mfma/run.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/mfma/trace -o run -- ./tools/mfma_gf 1024 > gpurun_out/mfma/trace.log 2>&1
rc=$?; echo "trace exit $rc"
cat gpurun_out/mfma/trace/*/run_kernel_stats.csv gpurun_out/mfma/trace/run_kernel_stats.csv 2>/dev/null | cut -c1-200
exit $rc
