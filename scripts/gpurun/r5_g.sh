#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/diag_render_batch.py > gpurun_out/r5_g_batch.log 2>&1; rc=$?
cat gpurun_out/r5_g_batch.log
exit $rc
