#!/bin/bash
# Profiles for profiles/<round>/ (run on the GPU box through gpurun):
#   1. rocprofv3 --kernel-trace --stats over the default bench command (the judged bench line itself);
#   2. two PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs, per MI355X_MICROARCH.md "rocprofv3 PMC slots")
#      over a short bench run, summarised per kernel by scripts/pmc_summary.py.
# Each GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
BENCH=${BENCH_ARGS:-""}
SHORT=${SHORT_ARGS:-"--steps 1 --pods-per-step 2000 --warmup 0 --no-cpu-baseline --kernel-iters 5"}
echo "== kernel trace: bench.py $BENCH"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 -u bench.py $BENCH > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; tail -2 $OUT/trace.log; [ $rc -eq 0 ] || exit $rc
for c in FETCH_SIZE WRITE_SIZE; do
  echo "== pmc $c: bench.py $SHORT"
  timeout -s KILL 120 rocprofv3 --pmc $c -d $OUT/pmc_$c -o run --output-format csv -- python3 -u bench.py $SHORT > $OUT/pmc_$c.log 2>&1
  rc=$?; echo "pmc $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 scripts/pmc_summary.py $OUT > $OUT/summary.txt && cat $OUT/summary.txt
