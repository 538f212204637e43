#!/bin/bash
# Round-3 diagnostic: per-kernel SQ / TCC counters of the exact-path kernels (xr_*) on a short bench run of one
# workload (WL, default c5).  One --pmc pass per counter group (rocprofv3 does not split passes).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
WL=${WL:-c5}
OUT=gpurun_out/r03/${TAG:-pmc_$WL}
mkdir -p $OUT
args="--workload $WL --steps 1 --pods-per-step ${PODS:-2000} --warmup 0 --no-cpu-baseline --kernel-iters 1 --check 0 --profile-pods 0 --single-pod-calls 0"
i=0
groups=("SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
        "SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_FLAT SQ_ACTIVE_INST_ANY"
        "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum")
[ -n "$GROUPS_N" ] && groups=("${groups[@]:0:$GROUPS_N}")
for grp in "${groups[@]}"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp -d $OUT/p$i -o run --output-format csv -- python3 -u bench.py $args > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/p$i.log; exit $rc; }
done
python3 scripts/pmc_kernels.py $OUT
