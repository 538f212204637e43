#!/bin/bash
# Round-3: full GPU suite (exclusive policies, wave-cooperative Reserve), xr stamps, c5 / shipped / c4 bench lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
out=gpurun_out/r03/${TAG:-g5}
mkdir -p "$out"
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 3 "$out/$name.log" | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}
run tests 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread ${TESTS:-}
[ -n "$NOSTAMPS" ] || run stamps_c5 300 python3 -u scripts/stamps_xr.py c5 50000 3000
[ -n "$NOSTAMPS" ] || run stamps_shipped 300 python3 -u scripts/stamps_xr.py shipped 50000 2000
for w in ${BENCHES:-c5 shipped c4}; do
  run bench_$w 400 python3 -u bench.py --workload $w --steps 5 --cpu-seconds 4 --single-pod-calls 20
done
