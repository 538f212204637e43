#!/bin/bash
# C3 geometry sweep on the product library (bench.py --steps 2, live period decomposition per line)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05/${TAG:-geom}
rm -rf $OUT; mkdir -p $OUT
i=0
while IFS= read -r args; do
  i=$((i+1))
  timeout -k 10 240 python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --check 0 --single-pod-calls 0 --no-pcie $args \
    > $OUT/g$i.json 2> $OUT/g$i.err || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); p=d['roofline'].get('period') or {}; print(repr(sys.argv[2]), round(d['value']), 'eval', p.get('eval_us'), 'merge', p.get('merge_us'), 'res', p.get('resolver_active_us'), 'ppr', p.get('pods_per_round'))" $OUT/g$i.json "$args"
done <<< "${SWEEP}"
