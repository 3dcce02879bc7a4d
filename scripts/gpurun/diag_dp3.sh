cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out &&
timeout -k 10 300 python scripts/diag_dp3.py 1024 > gpurun_out/diag_dp3_1024.log 2>&1
