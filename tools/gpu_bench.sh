#!/bin/bash
# Bench round trip: default 1-GPU line (instance headline + validator object),
# a 2-rank rehearsal of `--gpus 2` over gloo on the one GPU, and cfg5.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 400 python bench.py ${BENCH_ARGS:---steps 5 --warmup 1} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench exit $rc"; tail -c 4000 gpurun_out/bench.log; echo
if fatal $rc || [ $rc -ne 0 ]; then exit $rc; fi
HBRBC_BENCH_REHEARSE=1 timeout -k 10 400 python bench.py --gpus 2 --steps 3 --warmup 1 --count 4096 --vcount 1024 --no-cpu > gpurun_out/bench_g2.log 2>&1
rc=$?; echo "rehearse exit $rc"; tail -c 3000 gpurun_out/bench_g2.log; echo
if fatal $rc || [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --config cfg5 --steps 3 --warmup 1 --no-cpu > gpurun_out/bench_cfg5.log 2>&1
rc=$?; echo "cfg5 exit $rc"; tail -c 3000 gpurun_out/bench_cfg5.log
exit $rc
