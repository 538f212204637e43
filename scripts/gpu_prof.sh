#!/bin/bash
# rocprofv3 kernel-trace summary of a bench run + one full-size bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ARGS=${BENCH_ARGS:-"--nodes 10000 --pods-per-step 10000 --steps 3 --no-cpu-baseline --kernel-iters 20"}
echo "== rocprof ($ARGS)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 -u bench.py $ARGS > gpurun_out/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -3 gpurun_out/prof.log; [ $rc -eq 0 ] || exit $rc
find gpurun_out/prof -name "*kernel_stats.csv" -exec cat {} \; | head -20
if [ -n "$FULL_ARGS" ]; then
  echo "== bench full ($FULL_ARGS)"
  timeout -k 10 600 python3 -u bench.py $FULL_ARGS > gpurun_out/bench_full.log 2>&1
  rc=$?; echo "full rc=$rc"; tail -3 gpurun_out/bench_full.log
fi
