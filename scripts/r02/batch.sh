#!/bin/bash
# Round-2 sweep: C3 bench at batch sizes (short runs, oracle check on).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/batch
mkdir -p $OUT
for b in ${BATCHES:-24 32 48 64}; do
  timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --batch $b ${BENCH_ARGS} > $OUT/b$b.json 2> $OUT/b$b.err
  rc=$?; echo "batch $b rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/b$b.err; exit $rc; }
  python3 -c "import json; d=json.load(open('$OUT/b$b.json')); print(d['value'], d['oracle_check'], d['device_rounds'], d['roofline']['live_ms'])"
done
