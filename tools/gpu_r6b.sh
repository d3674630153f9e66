#!/bin/bash
# Round 6, call b: instance step pipelines A/B (cfg2 with its encode+Merkle
# rate, cfg3 headline), the 128-B row alignment A/B, the state machine tests
# after the pair-flag change, and one TCC pass over the cfg3 sponge.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/r6b
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 600 python -u -m pytest tests/test_rbc_sim.py tests/test_sharded.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests exit $rc"; tail -3 $OUT/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
export HBRBC_JIT=load
summ() { grep '^{' $1 | tail -1 | python3 -c "
import json,sys; d=json.load(sys.stdin)
print('$2', 'value', d['value'], 'ms', d['ms_per_step'], 'frac', d['roofline']['frac'], 'stages', {k: round(v,2) for k,v in d['stages_ms_per_step'].items()})" | tee -a $OUT/summary.txt; }
for rep in 1 2; do
for P in 1 2; do
  timeout -k 10 300 python bench.py --config cfg2 --mode instances --ipipes $P --no-cpu --f4-checks 0 --detail $OUT/cfg2_p${P}_${rep}.json > $OUT/cfg2_p${P}_${rep}.log 2>&1
  rc=$?; if fatal $rc; then exit $rc; fi
  summ $OUT/cfg2_p${P}_${rep}.log "cfg2 pipes=$P rep=$rep"
  python3 -c "import json; d=json.load(open('$OUT/cfg2_p${P}_${rep}.json')); print('   encode+merkle', d.get('encode_merkle', {}).get('value'), d.get('encode_merkle', {}).get('stages_ms_per_step'))" 2>/dev/null | tee -a $OUT/summary.txt
done
done
for rep in 1 2; do
for P in 1 2; do
  timeout -k 10 300 python bench.py --mode instances --ipipes $P --no-leaf-reuse --no-cpu --f4-checks 0 > $OUT/cfg3_p${P}_${rep}.log 2>&1
  rc=$?; if fatal $rc; then exit $rc; fi
  summ $OUT/cfg3_p${P}_${rep}.log "cfg3 pipes=$P rep=$rep"
done
for A in 16 128; do
  HBRBC_ROW_ALIGN=$A timeout -k 10 300 python bench.py --mode instances --no-leaf-reuse --no-cpu --f4-checks 0 > $OUT/cfg3_a${A}_${rep}.log 2>&1
  rc=$?; if fatal $rc; then exit $rc; fi
  summ $OUT/cfg3_a${A}_${rep}.log "cfg3 align=$A rep=$rep"
done
done
for A in 16 128; do
  HBRBC_ROW_ALIGN=$A timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "leaf_hash_kernel" --output-format csv -d $OUT/pmc_tcc_a$A -o run -- python3 bench.py --mode instances --steps 1 --warmup 1 --no-cpu --no-verify --no-leaf-reuse --f4-checks 0 > $OUT/pmc_tcc_a$A.log 2>&1
  rc=$?; echo "pmc align $A exit $rc"; if fatal $rc; then exit $rc; fi
done
exit 0
