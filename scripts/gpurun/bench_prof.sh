# usage: bash scripts/gpurun/bench_prof.sh <tag>  -> gpurun_out/bench_<tag>.json.log,
#        gpurun_out/prof_<tag>/ (rocprofv3 --kernel-trace --stats of the same bench command)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out &&
timeout -k 10 420 python bench.py > gpurun_out/bench_$1.json.log 2> gpurun_out/bench_$1.err &&
timeout -k 10 480 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$1 -o run -- python3 bench.py > gpurun_out/bench_$1_under_rocprof.json.log 2> gpurun_out/prof_$1.err
