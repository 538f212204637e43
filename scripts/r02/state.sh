#!/bin/bash
# Round-2 state capture: the full GPU suite, then the default C3 bench line (oracle check on) and the C4 / C5
# lines.  Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/state
mkdir -p $OUT
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 3 "$OUT/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
[ -n "$SKIP_TESTS" ] || run tests 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
run bench_c3 600 python3 -u bench.py ${C3_ARGS}
[ -n "$ONLY_C3" ] && exit 0
run bench_c5 600 python3 -u bench.py --workload c5
run bench_c4 600 python3 -u bench.py --workload c4
