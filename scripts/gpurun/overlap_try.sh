cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out &&
timeout -k 10 400 python bench.py --no_cpu_baseline --steps 15 --warmup 3 --groups 2 > gpurun_out/ov_g2.json.log 2> gpurun_out/ov_g2.err &&
timeout -k 10 400 python bench.py --no_cpu_baseline --steps 15 --warmup 3 --groups 1 > gpurun_out/ov_g1.json.log 2> gpurun_out/ov_g1.err
