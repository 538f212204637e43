#!/bin/bash
# Round-3: wide pass without the f64 reciprocal columns (v_rcp_f64 + Newton, two-way lrs_mem correction): GPU suite,
# C3 bench, C3 roofline passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
out=gpurun_out/r03/${TAG:-g10}
mkdir -p "$out"
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 3 "$out/$name.log" | cut -c1-500
  [ $rc -eq 0 ] || exit $rc
}
[ -n "$NOTESTS" ] || run tests 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread ${TESTS:-}
for w in ${BENCHES:-c3}; do
  run bench_$w 400 python3 -u bench.py --workload $w ${BARGS:-}
done
[ -n "$NOROOF" ] || WL=c3 bash scripts/r03/roofline.sh
