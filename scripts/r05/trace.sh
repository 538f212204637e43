#!/bin/bash
# Kernel trace of a short C3 run at depth ${DEPTH:-2} (args: extra bench args) + per-round timeline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05/${TAG:-trace}
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/t -o run --output-format csv -- python3 -u bench.py --steps 1 \
  --pods-per-step 20000 --warmup 1 --no-cpu-baseline --check 0 --profile-pods 0 --kernel-iters 1 --single-pod-calls 0 \
  --no-pcie "$@" > $OUT/bench.log 2>&1
rc=$?; echo "trace rc=$rc"; tail -2 $OUT/bench.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
python3 scripts/timeline.py $OUT/t ${DEPTH:-2} | tee $OUT/timeline.txt
find $OUT -name "*kernel_trace.csv" -size +20M -delete
