#!/bin/bash
# Round-3 C3 round-geometry sweep (pods per eval wave x round size x pipeline depth), throughput + live kernel times.
# No oracle check / CPU baseline (placements do not depend on the geometry; the GPU suite pins them).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
out=gpurun_out/r03/${TAG:-sweep}
mkdir -p "$out"
for cfg in ${CFGS:-"8 32 2" "4 32 2" "2 32 2" "4 32 3" "4 48 2" "8 64 2" "4 64 2" "4 32 4"}; do
  set -- $cfg
  name="ppw$1_b$2_d$3"
  echo "== $name"
  timeout -k 10 300 python3 -u bench.py --steps 3 --no-cpu-baseline --check 0 --single-pod-calls 0 \
    --pods-per-wave $1 --batch $2 --depth $3 ${BENCH_ARGS:-} > "$out/$name.json" 2> "$out/$name.err"
  rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || { tail -n 5 "$out/$name.err"; exit $rc; }
  python3 -c "import json,sys;d=json.loads(open('$out/$name.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$name', round(d['value']), r.get('live_ms'), r.get('isolated_ms'))"
done
