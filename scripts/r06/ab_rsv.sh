#!/bin/bash
# A/B of exact-pass library builds on the per-pod pass workloads (stock, c5r) plus the NUMA micro (scripts/micro).
# usage: LIBS="ab/libkg_rf.so koordinator_amd/libkoordgpu.so" ab_rsv.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06/ab
if [ -n "${MICRO:-}" ]; then
  timeout -k 10 120 python3 -u scripts/micro/numa_eval.py $MICRO > gpurun_out/r06/ab/micro.txt 2>&1
  rc=$?; cat gpurun_out/r06/ab/micro.txt; [ $rc -eq 0 ] || exit $rc
fi
for lib in ${LIBS:-}; do
  tag=$(basename $lib .so)
  for wl in ${WLS:-stock}; do
    KOORDGPU_LIB=$PWD/$lib timeout -k 10 ${T:-240} python3 -u bench.py --workload $wl --no-cpu-baseline --no-pcie \
      --single-pod-calls 0 ${EXTRA:-} > gpurun_out/r06/ab/${wl}_$tag.json 2> gpurun_out/r06/ab/${wl}_$tag.err
    rc=$?; [ $rc -eq 0 ] || { echo "$wl $tag rc=$rc"; tail -5 gpurun_out/r06/ab/${wl}_$tag.err; exit $rc; }
    python3 - gpurun_out/r06/ab/${wl}_$tag.json "$wl $tag" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], f"{d['value']:.0f}", "check", d.get("oracle_check"), d.get("oracle_check_pods"),
      "dominant", d["roofline"].get("kernel"), {k: round(v * 1e3, 2) for k, v in d["roofline"]["live_ms"].items()})
PY
  done
done
