#!/bin/bash
# Full GPU test suite, then C5 (DeviceShare) evidence: bench line with oracle check + CPU baseline, rocprof trace;
# then the default C3 bench line (regression check).  Stops at the first failing step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/c5
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/c5/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 4 "gpurun_out/c5/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
run smoke 240 python -u -c "import __graft_entry__ as g; g.smoke()"
run tests 900 python -u -m pytest tests -x -v -m "gpu and not slow" --timeout 120 --timeout-method thread
run bench_c5 500 python3 -u bench.py --workload c5 --check 2000
run trace_c5 400 rocprofv3 --kernel-trace --stats -d gpurun_out/c5/trace -o run --output-format csv -- python3 -u bench.py --workload c5 --no-cpu-baseline
run bench_c3 500 python3 -u bench.py --no-cpu-baseline
