#!/bin/bash
# default bench without the CPU leg (tag $1)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 500 python3 -u bench.py --no_cpu_baseline > gpurun_out/bench_$1.json.log 2> gpurun_out/bench_$1.err
