#!/bin/bash
# NUMA resolver pruning check: NUMA parity tests, then the C4 bench (oracle-checked).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r04/c4 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_numa_gpu.py tests/test_shipped_profile.py -x -q -m gpu --timeout 300 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/r04/c4/tests.log 2>&1
rc=$?; tail -n 3 gpurun_out/r04/c4/tests.log; [ $rc -eq 0 ] || exit $rc
for k in 1 2; do
  timeout -k 10 400 python3 -u bench.py --workload c4 --steps 5 --cpu-seconds 2 --single-pod-calls 0 > gpurun_out/r04/c4/bench$k.log 2>&1
  rc=$?; grep '^{"metric"' gpurun_out/r04/c4/bench$k.log | cut -c1-260; [ $rc -eq 0 ] || exit $rc
done
