#!/bin/bash
# C3 geometry sweep (depth x batch x pods-per-wave), short benches without CPU baseline / oracle check.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/sweep
mkdir -p $OUT
for g in "$@"; do
  set -- $g
  timeout -k 10 120 python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --check 0 --kernel-iters 2 \
    --profile-pods 10000 --depth $1 --batch $2 --pods-per-wave $3 > $OUT/b_$1_$2_$3.json 2> $OUT/b_$1_$2_$3.err
  rc=$?; [ $rc -eq 0 ] || { tail -3 $OUT/b_$1_$2_$3.err; exit $rc; }
  python3 -c "import json,sys; d=json.load(open('$OUT/b_$1_$2_$3.json')); r=d['roofline']; print('depth $1 B $2 ppw $3: %.0f pods/s' % d['value'], {k: round(v*1e3,1) for k,v in r['live_ms'].items()})"
done
