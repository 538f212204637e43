#!/bin/bash
# Round-3: shipped-profile test + bench lines for shipped / C2 / C1 (+ single-pod call latency at C3).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
out=gpurun_out/r03/${TAG:-bench}
mkdir -p "$out"
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 2 "$out/$name.log" | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}
run tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_shipped_profile.py
run shipped 600 python3 -u bench.py --workload shipped --steps 3 --cpu-seconds 6
run c2 400 python3 -u bench.py --workload c2 --cpu-seconds 6
run c1 300 python3 -u bench.py --workload c1 --cpu-seconds 4
run c3 600 python3 -u bench.py --steps 3 --no-cpu-baseline --check 2000
