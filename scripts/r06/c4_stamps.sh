#!/bin/bash
# C4: a fixture-checked bench line (50k pods = the committed fixture) and the NUMA resolver's per-pod stamps (dev build).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
timeout -k 10 400 python3 -u bench.py --workload c4 --steps 5 --warmup 1 --single-pod-calls 50 \
  > gpurun_out/r06/bench_c4.json 2> gpurun_out/r06/bench_c4.err || { tail -5 gpurun_out/r06/bench_c4.err; exit 1; }
tail -c 600 gpurun_out/r06/bench_c4.json
STAMPS_LIB=libkoordgpu_dev.so timeout -k 10 300 python3 -u scripts/stamps_numa.py 10000 4000 16 > gpurun_out/r06/stamps_c4.txt 2>&1
rc=$?; head -60 gpurun_out/r06/stamps_c4.txt; exit $rc
