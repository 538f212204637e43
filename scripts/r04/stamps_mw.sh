cd $GRAFT_REPO_ROOT && timeout -k 5 120 python -u scripts/r04/stamps_mw.py 100000 20000 ${DEPTH:-2}
