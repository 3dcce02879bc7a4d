cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out &&
timeout -k 10 600 python scripts/bench_policy.py DiffusionPolicy --num_envs 2048 --steps 48 --warmup 24 > gpurun_out/bench_dp.log 2>&1
