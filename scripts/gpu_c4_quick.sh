set -o pipefail
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_numa_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/numa_tests.log 2>&1; rc=$?; tail -2 gpurun_out/numa_tests.log; [ $rc -eq 0 ] || exit $rc
SWEEP="32:1 32:4 16:1" STEPS=2 bash scripts/gpu_c4_sweep.sh
