#!/bin/bash
# Round-3: full GPU suite, then bench lines (C3 default, C1, C2, shipped) with oracle checks.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
out=gpurun_out/r03/${TAG:-full}
mkdir -p "$out"
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 2 "$out/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
run tests 1100 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
for w in ${BENCHES:-c3 c1}; do
  run bench_$w 600 python3 -u bench.py --workload $w ${BENCH_ARGS:-}
done
