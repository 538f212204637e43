#!/bin/bash
# Round-3: kernel trace of a short exact-profile bench (WL, default c5) and the idle gaps between kernels.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
wl=${WL:-c5}
OUT=gpurun_out/r03/trace_$wl
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/t -o run --output-format csv -- python3 -u bench.py --workload $wl \
  --steps 1 --pods-per-step ${PODS:-3000} --warmup 1 --no-cpu-baseline --check 0 --profile-pods 0 --kernel-iters 1 \
  --single-pod-calls 0 > $OUT/bench.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/bench.log; exit $rc; }
python3 scripts/gaps.py $OUT/t xr_eval | tee $OUT/gaps.txt
