#!/bin/bash
# Round-2 diagnostic: SQ instruction / cycle counters per kernel on a short C3 run (one --pmc pass, 8 SQ counters).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/sq
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU \
  -d $OUT/pmc -o run --output-format csv -- python3 -u bench.py --steps 1 --pods-per-step 2000 --warmup 0 --no-cpu-baseline \
  --kernel-iters 2 --check 0 --profile-pods 0 ${BENCH_ARGS} > $OUT/run.log 2>&1
rc=$?; echo "pmc rc=$rc"; tail -3 $OUT/run.log; exit $rc
