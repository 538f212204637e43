#!/bin/bash
# C5 Reservation evidence: bench line (oracle check + CPU baseline), kernel trace (rocprofv3 --kernel-trace --stats).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/c5r
timeout -k 10 300 python -u -m pytest tests/test_reservation_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/c5r/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/c5r/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python3 -u bench.py --workload c5r --check 1500 > gpurun_out/c5r/bench.json 2> gpurun_out/c5r/bench.err
rc=$?; echo "bench_c5r rc=$rc"; tail -1 gpurun_out/c5r/bench.json | cut -c1-600; [ $rc -eq 0 ] || { tail -20 gpurun_out/c5r/bench.err; exit $rc; }
export KG_RSV_NO_GRAPH=1  # rocprofv3 kernel tracing crashes on graph launches of this path
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/c5r/trace -o run --output-format csv -- python3 -u bench.py --workload c5r --no-cpu-baseline --steps 3 > gpurun_out/c5r/trace.log 2>&1
rc=$?; echo "trace_c5r rc=$rc"; [ $rc -eq 0 ] || exit $rc
find gpurun_out/c5r/trace -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/c5r/kernel_stats.csv
head -8 gpurun_out/c5r/kernel_stats.csv | cut -c1-200
