#!/bin/bash
# round 4 records: the default bench under rocprofv3 --kernel-trace --stats (timed-window summary),
# then the HBM-traffic PMC passes of the GEMM and the fused Winograd kernel
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
bash scripts/gpurun/r3_benchprof.sh r4e || exit 1
bash scripts/gpurun/gemm_pmc.sh r4e || exit 1
bash scripts/gpurun/wino_pmc.sh r4e f4 || exit 1
find gpurun_out -name "*_kernel_trace.csv" -size +20M -delete
