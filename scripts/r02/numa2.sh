#!/bin/bash
# Round-2: NUMA resolver stamps (dev lib), the NUMA parity suites on the product lib, then a C4 line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/numa
mkdir -p $OUT
KOORDGPU_LIB=$PWD/koordinator_amd/libkoordgpu_dev.so timeout -k 10 120 python3 -u scripts/stamps_numa.py 10000 4000 16 \
  > $OUT/stamps.log 2>&1
rc=$?; head -22 $OUT/stamps.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_numa_gpu.py tests/test_numa_amplify.py} -x -q --timeout 300 \
  --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 5 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u bench.py --workload c4 --steps 3 --no-cpu-baseline > $OUT/c4.json 2> $OUT/c4.err
rc=$?; echo "c4 rc=$rc"; tail -2 $OUT/c4.err; cat $OUT/c4.json; exit $rc
