cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out &&
timeout -k 10 600 python scripts/prof_ffn_layout.py > gpurun_out/ffn_layout.log 2>&1
