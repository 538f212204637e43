#!/bin/bash
# Round-3: C3 resolver eager settle of staged rows + wide-pass pod staging in LDS: GPU suite, C3 stamps, C3 bench,
# C3 kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
out=gpurun_out/r03/${TAG:-g8}
mkdir -p "$out"
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 3 "$out/$name.log" | cut -c1-600
  [ $rc -eq 0 ] || exit $rc
}
[ -n "$NOTESTS" ] || run tests 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread ${TESTS:-}
run stamps_c3 300 python3 -u scripts/stamps.py 100000 20000 2 32
for w in ${BENCHES:-c3}; do
  run bench_$w 400 python3 -u bench.py --workload $w --steps ${STEPS:-10} --cpu-seconds 4 --single-pod-calls 20
done
SHORT="--workload c3 --steps 1 --pods-per-step 8000 --warmup 0 --no-cpu-baseline --check 0 --profile-pods 0 --kernel-iters 2 --single-pod-calls 0 --no-pcie"
run trace_c3 300 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- python3 -u bench.py $SHORT
python3 scripts/trace_summary.py $out/trace 2>/dev/null | head -12 || true
