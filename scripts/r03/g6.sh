#!/bin/bash
# Round-3: exact-round kernel gaps (c5, shipped), C3 resolver stamps, C3 roofline evidence (trace + PMC + SQ).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r03/g6
WL=c5 bash scripts/r03/trace_xr.sh || exit $?
WL=shipped PODS=1500 bash scripts/r03/trace_xr.sh || exit $?
timeout -k 10 300 python3 -u scripts/stamps.py 100000 20000 2 32 > gpurun_out/r03/g6/stamps_c3.log 2>&1 || exit $?
tail -n 34 gpurun_out/r03/g6/stamps_c3.log
[ -n "$NOROOF" ] || WL=c3 bash scripts/r03/roofline.sh
