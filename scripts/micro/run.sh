#!/bin/bash
cd "${GRAFT_REPO_ROOT}/scripts/micro"
export TMPDIR=/tmp
timeout -k 10 60 ./launch_costs && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d ../../gpurun_out/micro -o micro --output-format csv -- ./launch_costs > ../../gpurun_out/micro.log 2>&1; echo rc=$?
cat ../../gpurun_out/micro/*kernel_stats.csv
