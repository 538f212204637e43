#!/bin/bash
# Round-2 sweep: C3 bench at pipeline depths 2..4 (short runs, oracle check on).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/depth
mkdir -p $OUT
for d in ${DEPTHS:-2 3 4}; do
  timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --depth $d ${BENCH_ARGS} > $OUT/d$d.json 2> $OUT/d$d.err
  rc=$?; echo "depth $d rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/d$d.err; exit $rc; }
  python3 -c "import json; d=json.load(open('$OUT/d$d.json')); print(d['value'], d['oracle_check'], d['device_rounds'], d['roofline']['live_ms'])"
done
