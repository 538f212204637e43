#!/bin/bash
# Round-3: gloo two-process engine test + loopback + parity suites, then a C3 bench line (oracle-checked).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
out=gpurun_out/r03/${TAG:-g3}
mkdir -p "$out"
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 4 "$out/$name.log" | cut -c1-600
  [ $rc -eq 0 ] || exit $rc
}
run tests 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu ${TESTS:-tests/test_dist_engine_gloo.py tests/test_multirank_loopback.py tests/test_parity_gpu.py}
run bench_c3 600 python3 -u bench.py --steps 5 --no-cpu-baseline --check 10000 --single-pod-calls 50
