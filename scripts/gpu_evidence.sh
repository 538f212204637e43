#!/bin/bash
# Evidence refresh: C5 bench line (oracle check + CPU baseline) + kernel trace, then the default C3 bench line
# with its rocprof trace and PMC passes (gpu_bench.sh → gpu_prof.sh).  Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ev
timeout -k 10 600 python3 -u bench.py --workload c5 --check 2000 > gpurun_out/ev/bench_c5.json 2> gpurun_out/ev/bench_c5.err
rc=$?; echo "bench_c5 rc=$rc"; tail -1 gpurun_out/ev/bench_c5.json | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/ev/trace_c5 -o run --output-format csv -- python3 -u bench.py --workload c5 --no-cpu-baseline --steps 3 > gpurun_out/ev/trace_c5.log 2>&1
rc=$?; echo "trace_c5 rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_bench.sh
