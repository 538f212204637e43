#!/bin/bash
# C4 (NodeNUMAResource) evidence: geometry sweep, bench line with oracle check + CPU baseline, rocprof trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/c4
SWEEP="${SWEEP:-32:8 32:2 32:1 16:4}" bash scripts/gpu_c4_sweep.sh || exit $?
echo "== bench c4 (check + cpu baseline)"
timeout -k 10 400 python3 -u bench.py --workload c4 ${C4_ARGS:-} --check 2000 > gpurun_out/c4/bench.json 2> gpurun_out/c4/bench.err
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/c4/bench.err; cat gpurun_out/c4/bench.json; [ $rc -eq 0 ] || exit $rc
echo "== rocprof trace c4"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/c4/trace -o run --output-format csv -- python3 -u bench.py --workload c4 ${C4_ARGS:-} --no-cpu-baseline > gpurun_out/c4/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; tail -2 gpurun_out/c4/trace.log; exit $rc
