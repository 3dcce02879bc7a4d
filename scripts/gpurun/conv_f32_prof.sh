# f32 layer-1 conv profile only
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out &&
timeout -k 10 200 python scripts/prof_conv_f32.py 1024 > gpurun_out/conv_f32_prof_$1.log 2>&1
