#!/bin/bash
# Round 3u: rolled edge-chunk loop in the fused unframe (smaller reconstruct
# kernels).  Unframe/decode parity tests, then cfg3 (instances) fused vs
# unfused, then the default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_unframe_fused.py tests/test_gpu_parity.py > gpurun_out/r3u_tests.log 2>&1
rc=$?; echo "tests exit $rc"; if [ $rc -ne 0 ]; then exit $rc; fi
for f in 1 0; do
  HBRBC_JIT=load HBRBC_UNFRAME_FUSED=$f timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu --mode instances --f4-checks 0 > gpurun_out/r3u_cfg3_f$f.log 2>&1
  rc=$?; echo "cfg3 fused=$f exit $rc"; if fatal $rc; then exit $rc; fi
done
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/r3u_bench.log 2>&1
rc=$?; echo "bench exit $rc"
exit $rc
