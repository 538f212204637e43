#!/bin/bash
# Round-2 sweep: C3 at pods-per-wave values (eval waves per tile group), B=32, depth 2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/ppw
mkdir -p $OUT
for w in ${PPWS:-1 2 4 8}; do
  timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --pods-per-wave $w --check 4000 ${BENCH_ARGS} \
    > $OUT/w$w.json 2> $OUT/w$w.err
  rc=$?; echo "ppw $w rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/w$w.err; exit $rc; }
  python3 -c "import json; d=json.load(open('$OUT/w$w.json')); print(round(d['value']), d['oracle_check'], d['device_rounds'], {k: round(v*1e3,1) for k,v in d['roofline']['live_ms'].items()})"
done
