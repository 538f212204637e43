cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r04
timeout -k 5 120 python -u scripts/r04/stamps_mw.py 100000 20000 ${DEPTH:-2} > gpurun_out/r04/stamps.txt 2>&1; head -n 14 gpurun_out/r04/stamps.txt
export KOORDGPU_LIB=$GRAFT_REPO_ROOT/koordinator_amd/libkoordgpu_pf15.so
for dp in 2 3; do timeout -k 5 120 python -u scripts/r04/mw_diag.py 100000 40000 $dp || exit 1; done
