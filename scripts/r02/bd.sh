#!/bin/bash
# Round-2 sweep: C3 at (batch, depth) pairs with D·B ≤ 64 (one register bank of modified rows).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/bd
mkdir -p $OUT
for bd in ${PAIRS:-"32 2" "21 3" "16 4" "24 2" "40 1"}; do
  set -- $bd
  timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --batch $1 --depth $2 --check 4000 \
    > $OUT/b$1_d$2.json 2> $OUT/b$1_d$2.err
  rc=$?; echo "batch $1 depth $2 rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/b$1_d$2.err; exit $rc; }
  python3 -c "import json; d=json.load(open('$OUT/b$1_d$2.json')); print(round(d['value']), d['oracle_check'], d['device_rounds'], {k: round(v*1e3,1) for k,v in d['roofline']['live_ms'].items()})"
done
