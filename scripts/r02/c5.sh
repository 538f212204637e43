#!/bin/bash
# Round-2: GPU parity of C5 as one profile (Reservation + DeviceShare + ElasticQuota) and the quota / reservation
# suites it touches, then the combined bench line with the oracle check.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/c5
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_c5_combined.py tests/test_elasticquota.py tests/test_reservation_gpu.py tests/test_deviceshare_gpu.py} \
  -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|ERROR|SKIP" $OUT/tests.log | tail -n 40; tail -n 30 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u bench.py --workload c5 ${BENCH_ARGS:---steps 3 --no-cpu-baseline} > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; tail -n 3 $OUT/bench.err; cat $OUT/bench.json; exit $rc
