#!/bin/bash
# Round 6: the GPU suite (minus the 1M-pod fixture test unless FULL=1), new tests first.  Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
SEL=${SEL:-"gpu"}
K=${K:-"not c3_full_size"}
FILES=${FILES:-"tests"}
timeout -k 10 ${T:-1000} python -u -m pytest $FILES -x -v -m "$SEL" -k "$K" --timeout 300 --timeout-method thread \
  > gpurun_out/r06/${NAME:-gpu_tests}.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -n 30 gpurun_out/r06/${NAME:-gpu_tests}.log
exit $rc
