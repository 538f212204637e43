cd $GRAFT_REPO_ROOT
export KOORDGPU_LIB=$GRAFT_REPO_ROOT/koordinator_amd/${DIAG_LIB:-libkoordgpu_pf15.so}
for v in ${RESOLVERS:-mw 1wave}; do for dp in ${DEPTHS:-2 3}; do KG_RESOLVER=$v timeout -k 5 120 python -u scripts/r04/mw_diag.py 100000 40000 $dp || exit 1; done; done
