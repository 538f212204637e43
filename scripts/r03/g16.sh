#!/bin/bash
# Round-3: NUMA resolver candidate prefetch (LDS-DMA) + resolver slot-record prefetch: GPU suite, C4 stamps, benches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
out=gpurun_out/r03/${TAG:-g16}
mkdir -p "$out"
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n ${TAILN:-3} "$out/$name.log" | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}
run tests 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
TAILN=8 STAMPS_LIB=libkoordgpu_stamps.so run stamps_c4 300 python3 -u scripts/stamps_numa.py 10000 4000 16
for w in ${BENCHES:-c4 c5 shipped}; do
  run bench_$w 400 python3 -u bench.py --workload $w --steps 5 --cpu-seconds 4 --single-pod-calls 20
done
