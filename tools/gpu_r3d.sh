#!/bin/bash
# Round 3d measurements: per-call drop-in latency with lane-per-sponge and
# pair-lane sponges, cfg2's leaf hash in both forms, and a
# kernel trace of the state machine rounds (validator-sharded objects).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
HBRBC_SPONGE_PAIR=0 timeout -k 10 300 python tools/bench_percall.py gpurun_out/r3_percall_lane.jsonl > gpurun_out/r3d_percall_lane.log 2>&1
rc=$?; echo "percall lane exit $rc"; if fatal $rc; then exit $rc; fi
timeout -k 10 300 python tools/bench_percall.py gpurun_out/r3_percall_pair.jsonl > gpurun_out/r3d_percall_pair.log 2>&1
rc=$?; echo "percall pair exit $rc"; if fatal $rc; then exit $rc; fi
for p in 0 1; do
  HBRBC_SPONGE_PAIR=$p HBRBC_JIT=load timeout -k 10 300 python bench.py --config cfg2 --mode instances --steps 3 --warmup 1 --f4-checks 0 --no-cpu > gpurun_out/r3d_cfg2_pair$p.log 2>&1
  rc=$?; echo "cfg2 pair=$p exit $rc"; if fatal $rc; then exit $rc; fi
done
TAG=r3d bash tools/gpu_sm_prof.sh > /dev/null
echo "prof exit $?"
