#!/bin/bash
# eval_round geometry A/B: 2 nodes per lane x 8 waves (4 or 3 waves/SIMD) vs the round-3 4 x 4; parity subset first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r04 || exit 1
export KOORDGPU_LIB=$PWD/koordinator_amd/libkoordgpu_pf15.so
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread \
  -k "round_shapes or pipeline_depths or synthetic or ties or unschedulable or edge_clusters or poisoned or c2_scale" \
  > gpurun_out/r04/evalnpt_tests.log 2>&1 || { tail -30 gpurun_out/r04/evalnpt_tests.log; exit 1; }
tail -2 gpurun_out/r04/evalnpt_tests.log
for v in pf15 pf15_w3 pf15_n4; do
  export KOORDGPU_LIB=$PWD/koordinator_amd/libkoordgpu_$v.so
  for dp in 2 3; do
    echo "lib=$v"; timeout -k 5 120 python -u scripts/r04/mw_diag.py 100000 40000 $dp || exit 1
  done
  echo "lib=$v c2"; timeout -k 5 120 python -u scripts/r04/mw_diag.py 10000 40000 2 || exit 1
done
STAMPS_LIB=libkoordgpu_dev.so timeout -k 5 120 python -u scripts/stamps.py 100000 20000 2 > gpurun_out/r04/stamps_npt2.txt 2>&1 || exit 1
sed -n 1,8p gpurun_out/r04/stamps_npt2.txt
