#!/bin/bash
# PodTopologySpread / InterPodAffinity device parity, then the full GPU suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r04 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_pod_groups.py -x -v -m gpu --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r04/groups_tests.log 2>&1
rc=$?; tail -n 25 gpurun_out/r04/groups_tests.log; [ $rc -eq 0 ] || exit $rc
[ -n "$FULL" ] || exit 0
bash scripts/r04/full_tests.sh
