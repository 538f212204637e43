#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r04 || exit 1
timeout -k 5 180 python -u scripts/stamps_xr.py c5 50000 3000 > gpurun_out/r04/stamps_xr_c5.txt 2>&1 || exit 1
timeout -k 5 180 python -u scripts/stamps_xr.py shipped 50000 2000 > gpurun_out/r04/stamps_xr_shipped.txt 2>&1 || exit 1
head -50 gpurun_out/r04/stamps_xr_c5.txt
