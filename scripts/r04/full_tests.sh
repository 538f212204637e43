#!/bin/bash
# Full GPU suite (no -x) on a fresh box, then smoke. Each step under its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r04/full_tests.log 2>&1
rc=$?
tail -n 30 gpurun_out/r04/full_tests.log
exit $rc
