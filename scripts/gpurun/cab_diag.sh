cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out &&
timeout -k 10 200 python scripts/diag_cabinet.py > gpurun_out/cab_diag.log 2>&1
