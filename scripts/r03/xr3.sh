#!/bin/bash
# Round-3: full GPU suite, xr_resolve stamps (c5, shipped), c5 / shipped / c5r bench lines, SQ counters of c5.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
out=gpurun_out/r03/${TAG:-xr3}
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
run stamps_c5 300 python3 -u scripts/stamps_xr.py c5 50000 3000
run stamps_shipped 300 python3 -u scripts/stamps_xr.py shipped 50000 2000
run stamps_c3 300 python3 -u scripts/stamps.py 100000 20000 2 32
for w in ${BENCHES:-c5 shipped c5r}; do
  run bench_$w 400 python3 -u bench.py --workload $w --steps 5 --cpu-seconds 4 --single-pod-calls 50
done
[ -n "$NOPMC" ] || TAG=${TAG:-xr3}/pmc_c5 WL=c5 GROUPS_N=2 timeout -k 10 600 bash scripts/r03/pmc_xr.sh > $out/pmc.log 2>&1
echo "pmc rc=$?"; tail -n 14 $out/pmc.log | cut -c1-700
