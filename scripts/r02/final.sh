#!/bin/bash
# Round-2 closing evidence: the full GPU suite, the C3 / C4 / C5 bench lines, and rocprofv3 kernel stats of C4.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/final
mkdir -p $OUT
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 2 "$OUT/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
run smoke 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")"
run tests 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
run bench_c4 600 python3 -u bench.py --workload c4
run bench_c3 600 python3 -u bench.py
run bench_c5 600 python3 -u bench.py --workload c5
run prof_c4 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o c4 -- python3 -u bench.py \
  --workload c4 --steps 3 --no-cpu-baseline
find $OUT/prof -name '*stats.csv'
