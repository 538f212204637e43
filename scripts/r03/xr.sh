#!/bin/bash
# Round-3: the exact-profile GPU tests (batched exact rounds), then the shipped / c5 bench lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
out=gpurun_out/r03/${TAG:-xr}
mkdir -p "$out"
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 3 "$out/$name.log" | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}
run tests 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread ${TESTS:-tests/test_c5_combined.py tests/test_reservation_gpu.py tests/test_shipped_profile.py tests/test_default_plugins.py tests/test_single_pod.py tests/test_reservation_restore.py tests/test_golden_reservation.py tests/test_unreserve.py}
for w in ${BENCHES:-shipped c5}; do
  run bench_$w 400 python3 -u bench.py --workload $w ${BENCH_ARGS:-}
done
