#!/bin/bash
# f4 occupancy A/B: the pairing kernels built at 4 / 2 / 1 waves per SIMD
# (libhbrbc.so, libhbrbc_w2.so, libhbrbc_w1.so: -DHB_PAIR_WPE), grouped
# (prepared) checks, and the pairing parity tests on each variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for L in libhbrbc.so libhbrbc_w2.so libhbrbc_w1.so; do
  HBRBC_LIB=$PWD/hbbft_amd/$L timeout -k 10 300 python -u -m pytest tests/test_pairing.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/f4wpe_tests_$L.log 2>&1
  rc=$?; echo "$L tests exit $rc"; [ $rc -ne 0 ] && exit $rc
  HBRBC_LIB=$PWD/hbbft_amd/$L timeout -k 10 300 python tools/bench_pairing.py --prepared --n 262144 --reps 3 > gpurun_out/f4wpe_$L.log 2>&1
  rc=$?; echo "$L bench exit $rc"; tail -c 600 gpurun_out/f4wpe_$L.log; echo
  [ $rc -ne 0 ] && exit $rc
done
exit 0
