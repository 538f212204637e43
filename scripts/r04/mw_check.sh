#!/bin/bash
# Look-ahead resolver: GPU parity suite, then C3 A/B against the single-wave resolver.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r04/mw_tests.log 2>&1
rc=$?; tail -n 5 gpurun_out/r04/mw_tests.log; [ $rc -eq 0 ] || exit $rc
for v in mw 1wave; do
  KG_RESOLVER=$v timeout -k 10 300 python -u bench.py --steps 4 --no-cpu-baseline --single-pod-calls 0 --no-pcie \
    > gpurun_out/r04/bench_c3_$v.json 2> gpurun_out/r04/bench_c3_$v.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/r04/bench_c3_$v.json'));print('$v', round(d['value']), d['oracle_check'], d['roofline']['live_ms'])"
done
