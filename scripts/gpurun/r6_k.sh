#!/bin/bash
# round-6: the fp32 bench alone (no bf16 secondary, no C3 line, no CPU leg) under
# rocprofv3 --kernel-trace --stats, for the per-inference kernel breakdown
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6k
O=gpurun_out/r6k
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no_cpu_baseline --no_bf16_secondary --no_c3_per_rank --steps 20 --warmup 5 > $O/bench_under_rocprof.json.log 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
find $O -name "*_kernel_trace.csv" -size +40M -delete
echo done
