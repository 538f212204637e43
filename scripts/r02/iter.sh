#!/bin/bash
# Round-2 iteration: parity of the Fit + LoadAware path, stamps at C3 size, a short C3 bench with the oracle check.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/iter
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py tests/test_elasticquota.py -x -q --timeout 120 \
  --timeout-method thread -k "not c3_full and not c2_scale" > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 5 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for cfg in ${STAMPS:-"100000 20000 1 32" "100000 20000 2 32" "100000 20000 3 32" "100000 20000 4 32"}; do :; done
for cfg in "100000 20000 1 32" "100000 20000 2 32" "100000 20000 3 32" "100000 20000 4 32" "100000 20000 2 64"; do
  timeout -k 10 120 python3 -u scripts/stamps.py $cfg > $OUT/s_${cfg// /_}.log 2>&1
  rc=$?; head -2 $OUT/s_${cfg// /_}.log; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 400 python3 -u bench.py --steps 5 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; tail -n 2 $OUT/bench.err; cat $OUT/bench.json; exit $rc
