# calibrated physics traffic (PMC), then the default bench and its rocprofv3 kernel-trace summary
# usage: bash scripts/gpurun/r2_measure.sh <tag>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/pmc_$1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_$1/pmc_fetch -o run -- python3 scripts/prof_physics.py --calib > gpurun_out/pmc_$1/fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_$1/pmc_write -o run -- python3 scripts/prof_physics.py --calib > gpurun_out/pmc_$1/write.log 2>&1 &&
timeout -k 10 420 python bench.py > gpurun_out/bench_$1.json.log 2> gpurun_out/bench_$1.err &&
timeout -k 10 480 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$1 -o run -- python3 bench.py --no_cpu_baseline > gpurun_out/bench_$1_under_rocprof.json.log 2> gpurun_out/prof_$1.err
