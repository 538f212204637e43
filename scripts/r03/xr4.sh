#!/bin/bash
# Round-3: exact-path suites, xr_resolve stamps with Reserve lane stamps (c5, shipped), c5 / shipped bench lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
out=gpurun_out/r03/${TAG:-xr4}
mkdir -p "$out"
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 3 "$out/$name.log" | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}
run tests 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread ${TESTS:-tests/test_c5_combined.py tests/test_reservation_gpu.py tests/test_shipped_profile.py tests/test_default_plugins.py tests/test_reservation_restore.py tests/test_golden_reservation.py tests/test_unreserve.py tests/test_multirank_loopback.py}
run stamps_c5 300 python3 -u scripts/stamps_xr.py c5 50000 3000
run stamps_shipped 300 python3 -u scripts/stamps_xr.py shipped 50000 2000
for w in ${BENCHES:-c5 shipped}; do
  run bench_$w 400 python3 -u bench.py --workload $w --steps 5 --cpu-seconds 4 --single-pod-calls 20
done
