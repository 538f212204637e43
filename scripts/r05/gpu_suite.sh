#!/bin/bash
# The whole -m gpu suite on the product library (log under gpurun_out/r05/<TAG>/tests.log), then optional extra steps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05/${TAG:-suite}
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 ${SUITE_TIMEOUT:-900} python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu ${TESTS:-tests} \
  > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; grep -E "FAILED|Error" $OUT/tests.log | head -5; exit $rc
