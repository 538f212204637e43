#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r04 || exit 1
export KOORDGPU_LIB=$PWD/koordinator_amd/libkoordgpu_pf15.so
export AMD_LOG_LEVEL=1
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -x -v -m gpu --timeout 120 --timeout-method thread \
  -k "c2_scale or eval_paths or empty_cluster or edge_clusters" -p no:cacheprovider > gpurun_out/r04/evalnpt_dbg.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed|Abort|error|:hip|HSA" gpurun_out/r04/evalnpt_dbg.log | head -30; exit $rc
