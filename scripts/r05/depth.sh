#!/bin/bash
# C3 pipeline-depth sweep (bench.py lines only): LIB = the library under test, DEPTHS = the depths.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05/${TAG:-depth}
rm -rf $OUT; mkdir -p $OUT
export KOORDGPU_LIB=$PWD/koordinator_amd/${LIB:-libkoordgpu_pf15.so}
for d in ${DEPTHS:-2 3 4}; do
  timeout -k 10 240 python3 -u bench.py --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --check 0 --single-pod-calls 0 \
    --no-pcie --depth $d ${BENCH_ARGS} > $OUT/bench_d$d.json 2> $OUT/bench_d$d.err || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d.get('roofline',{}).get('period'))" $OUT/bench_d$d.json $d
done
