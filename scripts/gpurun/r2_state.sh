# full GPU suite + smoke, then the default bench and its rocprofv3 kernel-trace summary
# usage: bash scripts/gpurun/r2_state.sh <tag>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out &&
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/full_tests_$1.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$1.log 2>&1 &&
timeout -k 10 420 python bench.py > gpurun_out/bench_$1.json.log 2> gpurun_out/bench_$1.err &&
timeout -k 10 480 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$1 -o run -- python3 bench.py --no_cpu_baseline > gpurun_out/bench_$1_under_rocprof.json.log 2> gpurun_out/prof_$1.err &&
for n in 64 256 1024; do timeout -k 10 120 python scripts/prof_physics.py $n > gpurun_out/phys_prof_$1_$n.log 2>&1 || exit $?; done
