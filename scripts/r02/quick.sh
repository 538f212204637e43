#!/bin/bash
# Round-2 iteration: GPU parity of the Fit + LoadAware path, then a short C3 bench with the oracle check.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/quick
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py tests/test_elasticquota.py -x -v --timeout 120 \
  --timeout-method thread -k "not c3_full and not c2_scale" > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 5 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u bench.py --steps 5 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; tail -n 3 $OUT/bench.err; cat $OUT/bench.json; exit $rc
