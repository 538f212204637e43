#!/bin/bash
# Round 6 bench lines: C3 as the driver runs it (--steps 20 --warmup 5: 2M pods, every placement checked against the
# committed fixture), C4 and shipped over their fixture-covered queues (5 steps), each with the CPU baseline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
for spec in ${SPECS:-"c3:20:5" "c4:5:1" "shipped:5:1"}; do
  IFS=: read wl steps warm <<< "$spec"
  timeout -k 10 ${T:-420} python3 -u bench.py --workload $wl --steps $steps --warmup $warm ${EXTRA:-} \
    > gpurun_out/r06/bench_$wl.json 2> gpurun_out/r06/bench_$wl.err
  rc=$?; echo "$wl rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r06/bench_$wl.err; exit $rc; }
  python3 - "$wl" <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/r06/bench_{sys.argv[1]}.json"))
r, c = d["roofline"], d.get("cpu_baseline") or {}
print(sys.argv[1], f"{d['value']:.0f} {d['unit']}", "oracle_check", d.get("oracle_check"), d.get("oracle_check_pods"),
      "frac", round(r["frac"], 4), "cpu", round(c.get("value", 0), 1))
PY
done
