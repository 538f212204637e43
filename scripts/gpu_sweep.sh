#!/bin/bash
# Parameter sweep of short C3 bench lines: SWEEP="batch:ppw batch:ppw ..."
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for bp in ${SWEEP:-32:2}; do
  b=${bp%%:*}; p=${bp##*:}
  timeout -k 10 200 python3 -u bench.py --steps 1 --pods-per-step ${PODS:-30000} --warmup 1 --no-cpu-baseline --kernel-iters 10 --batch $b --pods-per-wave $p ${BENCH_ARGS:-} > gpurun_out/sw_$b_$p.json 2> gpurun_out/sw.err
  rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/sw.err; exit $rc; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/sw_$b_$p.json').read().strip().splitlines()[-1])
print('B=$b ppw=$p pods/s', round(d['value']), 'rounds', d['device_rounds'], {k: round(v*1e3,2) for k,v in d['roofline']['kernels_ms'].items()})"
done
