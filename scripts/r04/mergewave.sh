#!/bin/bash
# merge_wave: parity on round shapes / depths (pf15 build), then A/B diag at C3 size (wave vs block merge) + stamps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r04 || exit 1
export KOORDGPU_LIB=$PWD/koordinator_amd/libkoordgpu_pf15.so
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread \
  -k "round_shapes or pipeline_depths or synthetic or ties or unschedulable or edge_clusters or poisoned or c2_scale" \
  > gpurun_out/r04/mergewave_tests.log 2>&1 || { tail -30 gpurun_out/r04/mergewave_tests.log; exit 1; }
tail -2 gpurun_out/r04/mergewave_tests.log
for m in wave block; do
  for dp in 2 3; do
    if [ $m = block ]; then export KG_MERGE=block; else unset KG_MERGE; fi
    echo "merge=$m"; timeout -k 5 120 python -u scripts/r04/mw_diag.py 100000 40000 $dp || exit 1
  done
done
unset KG_MERGE
STAMPS_LIB=libkoordgpu_dev.so timeout -k 5 120 python -u scripts/stamps.py 100000 20000 2 > gpurun_out/r04/stamps_mergewave.txt 2>&1 || exit 1
sed -n 1,20p gpurun_out/r04/stamps_mergewave.txt
