#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5_j_prof -o r5j --output-format csv -- \
  python3 -u scripts/prof_raster_probe.py > gpurun_out/r5_j.log 2>&1 || { echo "rc=$?"; tail -20 gpurun_out/r5_j.log; exit 1; }
grep "ms per" gpurun_out/r5_j.log
