#!/bin/bash
# Round-3: wave-uniform NUMA Reserve (scalar take_cpus): full GPU suite, C4 / shipped stamps and bench lines,
# then the C3 roofline evidence (trace + FETCH/WRITE + SQ passes).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
out=gpurun_out/r03/${TAG:-g7}
mkdir -p "$out"
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 3 "$out/$name.log" | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}
[ -n "$NOTESTS" ] || run tests 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread ${TESTS:-}
STAMPS_LIB=libkoordgpu_stamps.so run stamps_c4 300 python3 -u scripts/stamps_numa.py 10000 4000 16
run stamps_shipped 300 python3 -u scripts/stamps_xr.py shipped 50000 2000
for w in ${BENCHES:-c4 shipped}; do
  run bench_$w 400 python3 -u bench.py --workload $w --steps 5 --cpu-seconds 4 --single-pod-calls 20
done
[ -n "$NOROOF" ] || WL=c3 bash scripts/r03/roofline.sh
