#!/bin/bash
# GPU parity suite, then the look-ahead resolver's stamps and diagnostics (profile-15 builds), both resolvers.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r04/tests_iter.log 2>&1
rc=$?; tail -n 3 gpurun_out/r04/tests_iter.log; grep -E "FAILED|Error" gpurun_out/r04/tests_iter.log | head -5
[ $rc -eq 0 ] || exit $rc
timeout -k 5 120 python -u scripts/r04/stamps_mw.py 100000 20000 2 > gpurun_out/r04/stamps.txt 2>&1 || exit $?
head -n 14 gpurun_out/r04/stamps.txt
export KOORDGPU_LIB=$GRAFT_REPO_ROOT/koordinator_amd/libkoordgpu_pf15.so
for v in mw 1wave; do for dp in 2 3; do KG_RESOLVER=$v timeout -k 5 120 python -u scripts/r04/mw_diag.py 100000 40000 $dp || exit 1; done; done
