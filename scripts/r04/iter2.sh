#!/bin/bash
# 1wave resolver stamps (LDS pod reads) + diag of both resolvers at depth 2 and 3, C3 100k nodes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r04 || exit 1
KG_RESOLVER=1wave STAMPS_LIB=libkoordgpu_dev.so timeout -k 5 120 python -u scripts/stamps.py 100000 20000 2 \
  > gpurun_out/r04/stamps_1wave.txt 2>&1 || exit 1
sed -n 1,3p gpurun_out/r04/stamps_1wave.txt
export KOORDGPU_LIB=$PWD/koordinator_amd/libkoordgpu_pf15.so
for v in 1wave mw; do
  for dp in 2 3; do
    KG_RESOLVER=$v timeout -k 5 120 python -u scripts/r04/mw_diag.py 100000 40000 $dp || exit 1
  done
done
