#!/bin/bash
# Round-2 evidence: the full GPU suite, the default C3 bench line (oracle check, CPU baselines at 16 / 1 / nproc
# threads), C1 / C4 / C5 lines, then the kernel trace of the default bench and the FETCH_SIZE / WRITE_SIZE passes
# (scripts/gpu_prof.sh) into gpurun_out/prof.  Every GPU step has its own time limit; stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/evidence
mkdir -p $OUT
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 2 "$OUT/$name.log" | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}
[ -n "$SKIP_TESTS" ] || run tests 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
run bench_c3 600 python3 -u bench.py --cpu-nproc
run bench_c1 300 python3 -u bench.py --workload c1
run bench_c4 600 python3 -u bench.py --workload c4
run bench_c5 600 python3 -u bench.py --workload c5
[ -n "$SKIP_PROF" ] || bash scripts/gpu_prof.sh
