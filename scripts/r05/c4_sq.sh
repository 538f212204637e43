#!/bin/bash
# C4 NUMA resolver instruction mix: one SQ counter pass over a short C4 run (kernel trace first for the time split)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05/${TAG:-c4sq}
rm -rf $OUT; mkdir -p $OUT
SHORT="--workload c4 --steps 1 --pods-per-step 1600 --warmup 0 --no-cpu-baseline --check 0 --single-pod-calls 0 --no-pcie --profile-pods 0 --kernel-iters 1"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 -u bench.py $SHORT > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/trace.log; exit $rc; }
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $OUT/pmc_1 -o run --output-format csv -- python3 -u bench.py $SHORT > $OUT/pmc_1.log 2>&1
rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/pmc_1.log; exit $rc; }
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_FLAT SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU -d $OUT/pmc_2 -o run --output-format csv -- python3 -u bench.py $SHORT > $OUT/pmc_2.log 2>&1
rc=$?; echo "pmc2 rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/pmc_2.log; exit $rc; }
python3 scripts/pmc_kernels.py $OUT > $OUT/sq.txt; grep -E "resolve_round_numa|eval_round_numa" $OUT/sq.txt | cut -c1-900
grep -E "resolve_round_numa|eval_round_numa|merge" $OUT/trace/run_kernel_stats.csv | cut -c1-200
