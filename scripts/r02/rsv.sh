#!/bin/bash
# Round-2: reservation / C5 parity (cached group graph, exact short calls), then C5 lines at the default step and
# at small steps (8 pods per call: the online shape).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/rsv
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_reservation_gpu.py tests/test_c5_combined.py tests/test_unreserve.py \
  tests/test_elasticquota.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u bench.py --workload c5 --steps 3 --no-cpu-baseline > $OUT/c5.json 2> $OUT/c5.err
rc=$?; echo "c5 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u bench.py --workload c5 --steps 40 --pods-per-step 8 --profile-pods 0 --no-cpu-baseline \
  > $OUT/c5_small.json 2> $OUT/c5_small.err
rc=$?; echo "c5 small rc=$rc"; exit $rc
