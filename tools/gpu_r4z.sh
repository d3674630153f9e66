#!/bin/bash
# Round 4, call z: the cfg3 headline at 32768 instances per step -- kernel
# trace + stats of the instance line (the roofline's profiled source), then
# the full validation (GPU tests, smoke, default line, 2-rank rehearsal).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
OUT=$PWD/gpurun_out/prof_r4z_cfg3; mkdir -p $OUT
HBRBC_JIT=load timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --mode instances --no-leaf-reuse --f4-checks 0 > $OUT/trace.log 2>&1
rc=$?; echo "trace exit $rc"; tail -c 400 $OUT/trace.log; echo
if fatal $rc; then exit $rc; fi
TAG=r4z bash tools/gpu_round.sh
