#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=r2a_cfg3 bash tools/profile.sh || exit $?
TAG=r2a_cfg5 BENCH_ARGS="--config cfg5 --steps 3 --warmup 1 --no-cpu --mode instances" PMC_ARGS="--config cfg5 --steps 1 --warmup 1 --no-cpu --mode instances --no-verify" bash tools/profile.sh
