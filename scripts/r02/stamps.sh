#!/bin/bash
# Round-2 diagnostic: in-kernel phase stamps of the round kernels at C3 size (args: "nodes pods depth batch" ...).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/stamps
mkdir -p $OUT
for cfg in "$@"; do
  echo "== $cfg"
  timeout -k 10 120 python3 -u scripts/stamps.py $cfg > $OUT/s_${cfg// /_}.log 2>&1
  rc=$?; cat $OUT/s_${cfg// /_}.log; [ $rc -eq 0 ] || exit $rc
done
