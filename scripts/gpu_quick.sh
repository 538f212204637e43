#!/bin/bash
# Quick GPU iteration: parity tests, then short 100k-node bench lines for each PPW value, optional FETCH pass.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?; tail -2 gpurun_out/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/tests.log | head -20; exit $rc; }
for ppw in ${PPWS:-2}; do
  timeout -k 10 300 python3 -u bench.py --nodes ${NODES:-100000} --pods-per-step 20000 --steps 2 --no-cpu-baseline --kernel-iters 20 --pods-per-wave $ppw --batch ${BATCH:-32} > gpurun_out/q_$ppw.log 2>&1
  rc=$?; echo "ppw=$ppw rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/q_$ppw.log; exit $rc; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/q_$ppw.log').read().strip().splitlines()[-1]); print(round(d['value']), {k: round(v*1e3,2) for k,v in d['roofline']['kernels_ms'].items()})"
done
if [ -n "$FETCH" ]; then
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/qf -o run --output-format csv -- python3 -u bench.py --nodes ${NODES:-100000} --steps 1 --pods-per-step 2000 --warmup 0 --no-cpu-baseline --kernel-iters 5 --pods-per-wave ${PPWS%% *} > gpurun_out/qf.log 2>&1
  rc=$?; echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 scripts/pmc_summary.py gpurun_out/qf_root 2>/dev/null | true
  python3 - <<'PY'
import csv,glob,collections
acc=collections.defaultdict(list)
for f in glob.glob('gpurun_out/qf/**/*counter_collection.csv',recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r['Kernel_Name'][:40]].append(float(r['Counter_Value']))
for k,v in acc.items(): print(f"{k:40s} n={len(v)} fetch_x2={2*1024*sum(v)/len(v)/1e6:.2f} MB")
PY
fi
