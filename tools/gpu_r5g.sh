#!/bin/bash
# Round 5, call g: sub-batch streams on separate hardware queues, staggered
# (the FP4-MFMA study showed a leaf-hash launch and the XOR encoder on two
# streams with their own queues overlapping: 22.5 + 6.0 -> 25.8 ms), A/B
# against the one-stream default, same box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp HBRBC_JIT=load
OUT=gpurun_out/r5g
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
run() {  # tag, env, args
  env $2 timeout -k 10 300 python bench.py --mode instances --steps 8 --warmup 2 --no-cpu --f4-checks 0 --no-leaf-reuse --no-riders $3 > $OUT/$1.log 2>&1
  rc=$?; if fatal $rc; then echo "$1 exit $rc"; exit $rc; fi
  grep '^{' $OUT/$1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); s=d['stages_ms_per_step']; print('%-28s %7.2f GB/s %6.2f ms/step  leaf %5.1f enc %4.1f rec %4.1f' % ('$1', d['value'], d['ms_per_step'], s['leaf_hash'], s['encode'], s['reconstruct']))" | tee -a $OUT/ab.txt
}
for rep in 1 2; do
  run s1_q4_$rep "GPU_MAX_HW_QUEUES=4" "--streams 1"
  run s2stag_q8_$rep "GPU_MAX_HW_QUEUES=8" "--streams 2 --stagger"
  run s4stag_q8_$rep "GPU_MAX_HW_QUEUES=8" "--streams 4 --stagger"
  run s2_q8_$rep "GPU_MAX_HW_QUEUES=8" "--streams 2"
done
# queue mapping of the staggered 2-stream run with 8 queues
env GPU_MAX_HW_QUEUES=8 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace_s2stag -o run -- python3 bench.py --mode instances --steps 3 --warmup 1 --no-cpu --f4-checks 0 --no-leaf-reuse --no-riders --streams 2 --stagger > $OUT/trace.log 2>&1
rc=$?; echo "trace exit $rc"; if fatal $rc; then exit $rc; fi
python3 tools/queue_map.py $(find $OUT/trace_s2stag -name "*kernel_trace.csv") hbrbc > $OUT/queue_map.json; cat $OUT/queue_map.json
exit 0
