cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out &&
timeout -k 10 300 python scripts/bench_policy.py DiffusionPolicy3d --num_envs 1024 --steps 30 --warmup 10 > gpurun_out/bench_dp3.log 2>&1 &&
timeout -k 10 300 python scripts/bench_policy.py Mlp --num_envs 1024 --steps 30 --warmup 6 > gpurun_out/bench_mlp.log 2>&1 &&
timeout -k 10 420 python scripts/bench_policy.py DiffusionPolicy --num_envs 256 --steps 16 --warmup 8 > gpurun_out/bench_dp.log 2>&1
