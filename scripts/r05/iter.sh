#!/bin/bash
# r5 iteration: parity of the round engine with an iteration library, then fused vs unfused C3 timelines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
LIB=${LIB:-libkoordgpu_pf15.so}
OUT=gpurun_out/r05/${TAG:-iter}
rm -rf $OUT; mkdir -p $OUT
export KOORDGPU_LIB=$PWD/koordinator_amd/$LIB
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_parity_gpu.py \
  -k "${TESTS:-synthetic or round_shapes or depths or poisoned or ties or edge_clusters or empty_cluster or incremental or node_updates or c2_scale or c3_full}" \
  > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for f in ${FUSE:-1 0}; do
  KG_FUSE=$f TAG=r05_fuse$f DEPTH=${DEPTH:-2} bash scripts/r05/trace.sh ${BENCH_ARGS} > $OUT/trace_fuse$f.txt 2>&1 || exit 1
  echo "== KG_FUSE=$f"; grep -E "eval|merge|resolve|period" $OUT/trace_fuse$f.txt
done
