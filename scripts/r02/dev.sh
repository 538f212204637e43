#!/bin/bash
# Round-2 iteration on the dev library (Fit + LoadAware profile only): stamps at C3 size, then a short C3 bench
# with the oracle check.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/dev
mkdir -p $OUT
export KOORDGPU_LIB=$PWD/koordinator_amd/libkoordgpu_dev.so
timeout -k 10 120 env STAMPS_LIB=libkoordgpu_dev.so python3 -u scripts/stamps.py 100000 20000 0 32 > $OUT/stamps.log 2>&1
rc=$?; head -40 $OUT/stamps.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u bench.py --steps 5 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; tail -n 2 $OUT/bench.err; cat $OUT/bench.json; exit $rc
