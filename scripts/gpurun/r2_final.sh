# the default bench (with the CPU baseline leg) and its rocprofv3 kernel-trace summary
# usage: bash scripts/gpurun/r2_final.sh <tag>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out &&
timeout -k 10 600 python bench.py > gpurun_out/bench_$1.json.log 2> gpurun_out/bench_$1.err &&
timeout -k 10 480 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$1 -o run -- python3 bench.py --no_cpu_baseline > gpurun_out/bench_$1_under_rocprof.json.log 2> gpurun_out/prof_$1.err
