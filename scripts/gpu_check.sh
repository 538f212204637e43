#!/bin/bash
# One GPU-box pass: smoke → GPU tests → small bench. Stops at the first failing step (no retries).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
run smoke 240 python -u -c "import __graft_entry__ as g; g.smoke()"
run tests 900 python -u -m pytest tests -x -v -m "gpu and not slow" --timeout 120 --timeout-method thread
run bench_small 300 python -u bench.py --nodes 10000 --pods-per-step 10000 --steps 3 --no-cpu-baseline --kernel-iters 20
