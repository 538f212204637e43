#!/bin/bash
# Round-2: C4 batch sweep (pods per NUMA round), then a rocprofv3 kernel-stats run of the default C4 line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/c4sweep
mkdir -p $OUT
for b in 8 24 32; do
  timeout -k 10 300 python3 -u bench.py --workload c4 --steps 2 --batch $b --no-cpu-baseline --check 500 \
    > $OUT/b$b.json 2> $OUT/b$b.err
  rc=$?; echo "batch $b rc=$rc $(python3 -c "import json,sys; print(json.load(open('$OUT/b$b.json'))['value'])" 2>/dev/null)"
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o c4 -- python3 -u bench.py --workload c4 --steps 3 \
  --no-cpu-baseline > $OUT/prof.json 2> $OUT/prof.err
rc=$?; echo "prof rc=$rc"; find $OUT/prof -name '*kernel_stats.csv' | head -3; exit $rc
