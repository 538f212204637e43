#!/bin/bash
# Reservation-affinity selectors: the reservation GPU tests, then the full GPU suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r04 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_reservation_gpu.py tests/test_reservation_restore.py -x -v -m gpu \
  --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04/rsv_aff_tests.log 2>&1
rc=$?; tail -n 12 gpurun_out/r04/rsv_aff_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/r04/full_tests.sh
