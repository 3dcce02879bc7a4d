#!/bin/bash
# round 3: the default bench (no CPU leg) under rocprofv3 --kernel-trace --stats; per-kernel totals
# over the timed fp32 region, delimited by the spin-kernel markers bench.py launches with
# RMBX_TRACE_MARKERS=1
# usage: bash scripts/gpurun/r3_benchprof.sh <tag>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export RMBX_TRACE_MARKERS=1
timeout -k 10 480 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$1 -o run -- python3 bench.py --no_cpu_baseline --no_bf16_secondary > gpurun_out/bench_$1_under_rocprof.json.log 2> gpurun_out/prof_$1.err
rc=$?
python3 scripts/trace_window.py gpurun_out/prof_$1/run_kernel_trace.csv --marker spin_kernel --steps 30 --top 45 > gpurun_out/prof_$1_window.txt
find gpurun_out -name "*_kernel_trace.csv" -delete
exit $rc
