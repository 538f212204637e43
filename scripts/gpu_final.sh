#!/bin/bash
# Round-end evidence: full GPU suite (incl. slow), C3 default bench + rocprof trace + PMC passes (gpu_prof.sh),
# C4 and C5 bench lines with oracle checks + CPU baselines and their kernel traces.  Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/final
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/final/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 3 "gpurun_out/final/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
run tests 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
run bench_c3 600 python3 -u bench.py
run bench_c4 600 python3 -u bench.py --workload c4 --check 2000
run trace_c4 400 rocprofv3 --kernel-trace --stats -d gpurun_out/final/trace_c4 -o run --output-format csv -- python3 -u bench.py --workload c4 --no-cpu-baseline --steps 3
run bench_c5 600 python3 -u bench.py --workload c5 --check 2000
bash scripts/gpu_prof.sh
