#!/bin/bash
# C5 (DeviceShare) geometry sweep: SWEEP="B:ppw ..." → one short bench line each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for bp in ${SWEEP:-32:8 32:4 32:2 16:8}; do
  b=${bp%%:*}; p=${bp##*:}
  timeout -k 10 300 python3 -u bench.py --workload c5 --steps ${STEPS:-2} --batch $b --pods-per-wave $p --kernel-iters 10 \
    --no-cpu-baseline > gpurun_out/c5_sweep_${b}_${p}.json 2> gpurun_out/c5_sweep_${b}_${p}.err || exit $?
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/c5_sweep_${b}_${p}.json').read().strip().splitlines()[-1])
print('B=$b ppw=$p pods/s', round(d['value']), 'rounds', d['device_rounds'], {k: round(v*1e3,1) for k,v in d['roofline']['kernels_ms'].items()})"
done
