#!/bin/bash
# Round-3: roofline passes (trace + FETCH/WRITE + SQ) of the exact wide pass (xr_eval) for C5 and the shipped profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
WL=c5 PODS=6000 PROFPODS=6000 bash scripts/r03/roofline.sh || exit $?
WL=shipped PODS=2000 PROFPODS=2000 bash scripts/r03/roofline.sh || exit $?
