#!/bin/bash
# DeviceShare (C5 GPU-share part) on the GPU box: parity tests, then a short bench line with an oracle check.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ds
echo "== ds tests"
timeout -k 10 600 python -u -m pytest tests/test_deviceshare_gpu.py -x -v -m gpu --timeout 120 --timeout-method thread \
  > gpurun_out/ds/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 30 gpurun_out/ds/tests.log; [ $rc -eq 0 ] || exit $rc
echo "== bench c5"
timeout -k 10 400 python3 -u bench.py --workload c5 ${C5_ARGS:---steps 3 --no-cpu-baseline --kernel-iters 10} --check 1500 \
  > gpurun_out/ds/bench.json 2> gpurun_out/ds/bench.err
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/ds/bench.err; cat gpurun_out/ds/bench.json; exit $rc
