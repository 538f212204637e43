#!/bin/bash
# Per-kernel time of the stock profile's per-pod exact pass (plain launches so the trace sees every kernel).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04/stock_prof
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 300 python3 -u bench.py --workload stock --steps 3 --cpu-seconds 2 --single-pod-calls 0 > $OUT/bench.log 2>&1
rc=$?; tail -n 2 $OUT/bench.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
KG_RSV_NO_GRAPH=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
  python3 -u bench.py --workload stock --steps 1 --warmup 0 --no-cpu-baseline --check 0 --single-pod-calls 0 --no-pcie \
  > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/trace.log; exit $rc; }
find $OUT/trace -name "*kernel_stats.csv" -exec cut -d, -f1-8 {} \; | head -20
