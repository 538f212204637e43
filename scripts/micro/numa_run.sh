#!/bin/bash
# NUMA micro: the builds given in LIBS (results compared bit for bit), then PMC passes on the first (I-cache, issue)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06/micro
timeout -k 10 200 python3 -u scripts/micro/numa_eval.py $LIBS > gpurun_out/r06/micro/ab.txt 2>&1
rc=$?; cat gpurun_out/r06/micro/ab.txt; [ $rc -eq 0 ] || exit $rc
if [ -n "${PMC:-}" ]; then
  for lib in $LIBS; do
    tag=$(echo $lib | tr '/' '_')
    timeout -s KILL 90 rocprofv3 --pmc $PMC --kernel-trace --stats -d gpurun_out/r06/micro/pmc_$tag -o pmc --output-format csv \
      -- python3 -u scripts/micro/numa_eval.py $lib > gpurun_out/r06/micro/pmc_$tag.log 2>&1
    rc=$?; echo "pmc $lib rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/r06/micro/pmc_*/**/*counter_collection.csv", recursive=True)):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "")
        if "k_numa" in k:
            acc[k.split("(")[0]][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, c in sorted(acc.items()):
        print(f.split("/")[3], k, {n: int(v) for n, v in sorted(c.items())})
PY
fi
