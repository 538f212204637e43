#!/bin/bash
# Round-3 GPU check of the new / changed suites only (fast iteration).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
out=gpurun_out/r03/${TAG:-new}
mkdir -p "$out"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_topology_policy.py tests/test_golden_numa_score2.py tests/test_deviceshare_gpu.py \
  tests/test_reservation_restore.py tests/test_numa_amplify.py tests/test_fit_aux.py tests/test_shipped_profile.py \
  ${EXTRA:-} > "$out/tests.log" 2>&1
rc=$?; tail -n 25 "$out/tests.log"; exit $rc
