#!/bin/bash
# Round-2: multi-rank engine through the loopback test hook (G engines on one GPU), then the single-rank suites
# the sharding touched (DeviceShare rounds, Fit + LoadAware parity).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/multi
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest ${TESTS:-tests/test_multirank_loopback.py tests/test_deviceshare_gpu.py tests/test_parity_gpu.py} \
  -x -v --timeout 200 --timeout-method thread ${PYTEST_ARGS} > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|ERROR|SKIP" $OUT/tests.log | tail -n 40; tail -n 30 $OUT/tests.log; exit $rc
