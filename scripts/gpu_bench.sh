#!/bin/bash
# Default bench line (the judged configuration) then the rocprof trace + PMC passes (gpu_prof.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== bench (default)"
timeout -k 10 600 python3 -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.err; cat gpurun_out/bench.json; [ $rc -eq 0 ] || exit $rc
[ -n "$NO_PROF" ] && exit 0
bash scripts/gpu_prof.sh
