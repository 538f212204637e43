#!/bin/bash
# C3 geometry sweep (100k nodes): pipeline depth x round size, 3 steps each, no baselines.  Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
OUT=gpurun_out/r06/${NAME:-c3_sweep}.txt
: > $OUT
for cfg in ${CFGS:-"2:38" "3:38" "3:32" "3:44" "4:32" "2:40"}; do
  d=${cfg%%:*}; b=${cfg##*:}
  timeout -k 10 240 python3 -u bench.py --steps ${STEPS:-3} --warmup 1 --depth $d --batch $b --no-cpu-baseline --no-pcie \
    --single-pod-calls 0 --check 0 --profile-pods 5000 ${EXTRA:-} > gpurun_out/r06/sweep_one.json 2> gpurun_out/r06/sweep_one.err
  rc=$?
  [ $rc -eq 0 ] || { echo "depth $d batch $b rc=$rc"; tail -5 gpurun_out/r06/sweep_one.err; exit $rc; }
  python3 - "$d" "$b" >> $OUT <<'PY'
import json, sys
d = json.load(open("gpurun_out/r06/sweep_one.json"))
p = d["roofline"]["period"] or {}
print(f"depth {sys.argv[1]} B {sys.argv[2]}: {d['value']/1e3:.1f}k pods/s  period {p.get('us_per_round', 0):.1f} us/"
      f"{p.get('pods_per_round', 0):.2f} pods  resolver {p.get('resolver_active_us') or 0:.1f}  eval "
      f"{p.get('eval_us') or 0:.1f}  merge {p.get('merge_us') or 0:.1f}  slow {p.get('slow_pod_frac') or 0:.3f}")
PY
  tail -1 $OUT
done
