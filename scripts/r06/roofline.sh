#!/bin/bash
# Round-6 roofline evidence for the C3 wide pass (one workload geometry, one short command for every pass):
# kernel trace --stats, FETCH_SIZE / WRITE_SIZE passes (HBM traffic, gfx950-corrected by scripts/pmc_summary.py),
# two SQ counter passes (instruction mix, wave / busy / wait cycles) summarised by scripts/pmc_kernels.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
wl=${WL:-c3}
OUT=gpurun_out/r06/roofline_$wl
rm -rf $OUT; mkdir -p $OUT
SHORT="--workload $wl --steps 1 --pods-per-step ${PODS:-8000} --warmup 0 --no-cpu-baseline --check 0 --profile-pods ${PROFPODS:-8000} --kernel-iters 2 --single-pod-calls 0 --no-pcie"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 -u bench.py $SHORT > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/trace.log; exit $rc; }
# heartbeat: a PMC pass serialises every dispatch and writes its CSV only at exit
( while sleep 30; do echo "[roofline] $(date +%T) running"; done ) &
HB=$!
trap "kill $HB" EXIT
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" \
           "SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_FLAT SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $grp -d $OUT/pmc_$i -o run --output-format csv -- python3 -u bench.py $SHORT > $OUT/pmc_$i.log 2>&1
  rc=$?; echo "pmc $i ($grp) rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/pmc_$i.log; exit $rc; }
done
# pmc_summary.py reads pmc_FETCH_SIZE / pmc_WRITE_SIZE directories
mv $OUT/pmc_1 $OUT/pmc_FETCH_SIZE && mv $OUT/pmc_2 $OUT/pmc_WRITE_SIZE
META=$(python3 -c "import bench,json; n,_,b,p,_=bench.WORKLOADS['$wl']; print(json.dumps({'nodes':n,'batch_pods':b,'pods_per_wave':p,'depth':0,'workload':'$wl','command':'bench.py $SHORT'}))")
python3 scripts/pmc_summary.py $OUT "$META" > $OUT/summary.txt && cat $OUT/summary.txt
python3 scripts/pmc_kernels.py $OUT > $OUT/sq.txt && cat $OUT/sq.txt | cut -c1-600
find $OUT -name "*counter_collection.csv" -size +20M -delete
