#!/bin/bash
# Iteration loop on the GPU box: parity tests (stop at first failure), then a short C3 bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests -m "gpu and not slow" -x -q --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?; tail -3 gpurun_out/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/tests.log | head -30; exit $rc; }
timeout -k 10 300 python3 -u bench.py --steps ${STEPS:-3} --no-cpu-baseline --kernel-iters 20 ${BENCH_ARGS:-} > gpurun_out/iter_bench.json 2> gpurun_out/iter_bench.err
rc=$?; tail -2 gpurun_out/iter_bench.err; [ $rc -eq 0 ] || exit $rc
python3 -c "
import json; d=json.loads(open('gpurun_out/iter_bench.json').read().strip().splitlines()[-1])
print('pods/s', round(d['value']), 'ms/step', round(d['ms_per_step'],2), 'rounds', d['device_rounds'], {k: round(v*1e3,2) for k,v in d['roofline']['kernels_ms'].items()})"
