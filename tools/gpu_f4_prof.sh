#!/bin/bash
# f4 profiles: kernel trace + stats and one SQ counter pass over the pairing
# microbench (131072 checks), then tools/pmc_pairing.py -> ops per check.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/prof_f4
mkdir -p $OUT
N=${N:-262144}
PREP=${PREP---prepared}
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 tools/bench_pairing.py --n $N --reps 2 $PREP > $OUT/trace.log 2>&1
rc=$?; echo "trace exit $rc"; tail -2 $OUT/trace.log
if fatal $rc || [ $rc -ne 0 ]; then exit $rc; fi
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VMEM --output-format csv -d $OUT/pmc -o run -- python3 tools/bench_pairing.py --n $N --reps 1 $PREP > $OUT/pmc.log 2>&1
rc=$?; echo "pmc exit $rc"; tail -2 $OUT/pmc.log
if fatal $rc || [ $rc -ne 0 ]; then exit $rc; fi
python3 tools/pmc_pairing.py $OUT $N
