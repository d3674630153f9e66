#!/bin/bash
# Round-2 profile set: kernel trace + stats and the FETCH/WRITE/SQ counter
# passes for cfg3 (headline) and cfg5, each under gpurun_out/prof_<tag>.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG3:-r2b_cfg3} bash tools/profile.sh || exit $?
TAG=${TAG5:-r2b_cfg5} BENCH_ARGS="--config cfg5 --steps 3 --warmup 1 --no-cpu --mode instances" PMC_ARGS="--config cfg5 --steps 1 --warmup 1 --no-cpu --mode instances --no-verify" bash tools/profile.sh
