#!/bin/bash
# r5 resolver iteration: round-engine parity with the iteration library, then the C3 depth sweep.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05/${TAG:-pre}
rm -rf $OUT; mkdir -p $OUT
export KOORDGPU_LIB=$PWD/koordinator_amd/${LIB:-libkoordgpu_pf15.so}
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_parity_gpu.py \
  -k "${TESTS:-synthetic or round_shapes or depths or poisoned or ties or edge_clusters or empty_cluster or incremental or node_updates or c2_scale or c3_full}" \
  > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
TAG=${TAG:-pre}_depth DEPTHS="${DEPTHS:-2 3 4}" bash scripts/r05/depth.sh
