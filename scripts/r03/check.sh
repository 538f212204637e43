#!/bin/bash
# Round-3 state check: full GPU suite, then a C3 bench line (oracle-checked).  Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
out=gpurun_out/r03/${TAG:-check}
mkdir -p "$out"
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 3 "$out/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
run tests 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread ${TESTS:-}
[ -n "$NOBENCH" ] || run bench_c3 600 python3 -u bench.py --steps 5
