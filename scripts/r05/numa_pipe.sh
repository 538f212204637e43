#!/bin/bash
# r5: NUMA rounds pipelined — C4 parity on the iteration library, then the C4 bench at depths 1..3.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05/${TAG:-numa}
rm -rf $OUT; mkdir -p $OUT
export KOORDGPU_LIB=$PWD/koordinator_amd/${LIB:-libkoordgpu_pf15.so}
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_numa_gpu.py tests/test_numa_amplify.py tests/test_unreserve.py -k "${TESTS:-c4 or numa or amplif}" \
  > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for d in ${DEPTHS:-1 2 3}; do
  timeout -k 10 240 python3 -u bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline --check ${CHECK:-1000} \
    --single-pod-calls 0 --no-pcie --depth $d > $OUT/bench_d$d.json 2> $OUT/bench_d$d.err || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); p=d['roofline'].get('period') or {}; print(sys.argv[2], d['value'], p.get('us_per_round'), p.get('resolver_active_us'), d.get('check'))" $OUT/bench_d$d.json $d
done
