#!/bin/bash
# Round-3: exact-profile GPU tests after the xr_eval regrid, xr_resolve per-pod stamps (c5, shipped), bench lines,
# then the C3 round-geometry sweep.  Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
out=gpurun_out/r03/${TAG:-xr2}
mkdir -p "$out"
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 3 "$out/$name.log" | cut -c1-600
  [ $rc -eq 0 ] || exit $rc
}
run tests 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
run stamps_c5 300 python3 -u scripts/stamps_xr.py c5 50000 3000
run stamps_shipped 300 python3 -u scripts/stamps_xr.py shipped 50000 2000
for w in ${BENCHES:-c5 shipped}; do
  run bench_$w 400 python3 -u bench.py --workload $w --steps 5 --cpu-seconds 4 --single-pod-calls 50
done
[ -n "$NOSWEEP" ] || TAG=${TAG:-xr2}/sweep bash scripts/r03/sweep_c3.sh
DEPTH=2 timeout -k 10 400 bash scripts/r02/trace.sh > gpurun_out/r03/${TAG:-xr2}/trace.log 2>&1; echo "trace rc=$?"; tail -n 30 gpurun_out/r03/${TAG:-xr2}/trace.log
