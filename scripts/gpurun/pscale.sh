cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/pscale &&
for n in 1024 4096; do timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/pscale/n$n -o run -- python3 scripts/prof_physics.py $n > gpurun_out/pscale/n$n.log 2>&1 || exit 1; done
