#!/bin/bash
# Round-5 closing evidence for the committed source: full GPU suite, smoke, every bench line (oracle-checked), the
# C3 roofline passes (trace + FETCH/WRITE + SQ, live timing in the same process).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
out=gpurun_out/r05/${TAG:-final}
mkdir -p "$out"
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 3 "$out/$name.log" | cut -c1-500
  [ $rc -eq 0 ] || exit $rc
}
[ -n "$NOTESTS" ] || run tests 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread
run smoke 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run bench_c3 400 python3 -u bench.py
for w in ${BENCHES:-c2 c1 c5 c5r shipped c4}; do
  run bench_$w 400 python3 -u bench.py --workload $w --steps 5 --cpu-seconds 4 --single-pod-calls 20
done
[ -n "$NOROOF" ] || WL=c3 bash scripts/r05/roofline.sh
