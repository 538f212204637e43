#!/bin/bash
# Round-2 profiles: for each workload (WLS, default "c3 c4 c5 c5ds"), a kernel trace with --stats of a short bench
# run and two PMC passes (FETCH_SIZE, WRITE_SIZE: separate runs), summarised per kernel by scripts/pmc_summary.py
# with the workload geometry as _meta (bench.py matches it to fill roofline.traffic).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
for wl in ${WLS:-c3 c4 c5 c5ds}; do
  OUT=gpurun_out/pmc/$wl
  rm -rf $OUT; mkdir -p $OUT
  case $wl in
    c3) SHORT="--steps 1 --pods-per-step 20000";;
    c4) SHORT="--steps 1 --pods-per-step 2000";;
    c5ds) SHORT="--steps 1 --pods-per-step 3000";;
    *)  SHORT="--steps 1 --pods-per-step 400";;
  esac
  SHORT="--workload $wl $SHORT --warmup 0 --no-cpu-baseline --check 0 --profile-pods 0 --kernel-iters 2"
  echo "== $wl trace"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 -u bench.py $SHORT > $OUT/trace.log 2>&1
  rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/trace.log; exit $rc; }
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 200 rocprofv3 --pmc $c -d $OUT/pmc_$c -o run --output-format csv -- python3 -u bench.py $SHORT > $OUT/pmc_$c.log 2>&1
    rc=$?; echo "pmc $c rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/pmc_$c.log; exit $rc; }
  done
  META=$(python3 -c "import bench,json; n,_,b,p,_=bench.WORKLOADS['$wl']; print(json.dumps({'nodes':n,'batch_pods':b,'pods_per_wave':p,'depth':0,'workload':'$wl','command':'bench.py $SHORT'}))")
  python3 scripts/pmc_summary.py $OUT "$META" > $OUT/summary.txt && cat $OUT/summary.txt
  # keep only the summaries (the raw per-dispatch CSVs are large)
  find $OUT -name "*counter_collection.csv" -size +20M -delete
done
