#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/prof_gemm_presplit.py > gpurun_out/r5_p_prof.log 2>&1 || { echo "prof rc=$?"; tail -20 gpurun_out/r5_p_prof.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5_p_prof.log | grep -v "^group"
