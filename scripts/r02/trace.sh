#!/bin/bash
# Kernel trace of a short C3 bench (args: extra bench args), timeline per round.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/trace
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/t -o run --output-format csv -- python3 -u bench.py --steps 1 \
  --pods-per-step 20000 --warmup 1 --no-cpu-baseline --check 0 --profile-pods 0 --kernel-iters 1 "$@" > $OUT/bench.log 2>&1
rc=$?; echo "trace rc=$rc"; tail -2 $OUT/bench.log; [ $rc -eq 0 ] || exit $rc
python3 scripts/timeline.py $OUT/t ${DEPTH:-3}
