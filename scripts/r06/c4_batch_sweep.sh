#!/bin/bash
# C4 batch sweep with the two-wave NUMA resolver (depth 2: batch ≤ 30 keeps d·B < 62); every line fixture-checked.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06/c4_sweep
for b in ${BATCHES:-16 20 24 30}; do
  timeout -k 10 240 python3 -u bench.py --workload c4 --steps 5 --warmup 1 --batch $b --no-cpu-baseline --no-pcie \
    --single-pod-calls 0 > gpurun_out/r06/c4_sweep/b$b.json 2> gpurun_out/r06/c4_sweep/b$b.err
  rc=$?; [ $rc -eq 0 ] || { echo "b$b rc=$rc"; tail -3 gpurun_out/r06/c4_sweep/b$b.err; exit $rc; }
  python3 - gpurun_out/r06/c4_sweep/b$b.json $b <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("batch", sys.argv[2], round(d["value"]), "check", d.get("oracle_check"), d.get("oracle_check_pods"),
      "resolver us/round", round(d["roofline"]["period"]["resolver_active_us"], 1), "rounds", d["device_rounds"])
PY
done
