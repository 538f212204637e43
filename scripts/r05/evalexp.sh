#!/bin/bash
# eval_round timing A/B (bench live kernel timing; results of the experiment library are not checked)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05/${TAG:-evalexp}
rm -rf $OUT; mkdir -p $OUT
for lib in ${LIBS:-libkoordgpu_pf15.so libkoordgpu_exp.so}; do
  KOORDGPU_LIB=$PWD/koordinator_amd/$lib timeout -k 10 240 python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline \
    --check 0 --single-pod-calls 0 --no-pcie ${BENCH_ARGS} > $OUT/$lib.json 2> $OUT/$lib.err || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); p=d['roofline'].get('period') or {}; print(sys.argv[2], round(d['value']), 'eval', p.get('eval_us'), 'merge', p.get('merge_us'), 'res', p.get('resolver_active_us'))" $OUT/$lib.json $lib
done
