#!/bin/bash
# HBM traffic of the fp32-accurate GEMM kernel and the patch-staged convs over one fp32 ACT inference:
# FETCH_SIZE and WRITE_SIZE passes (tools/pmc_traffic.py --gemm / --convp reduce them)
# usage: bash scripts/gpurun/gemm_pmc.sh <tag>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/gemm_pmc_$1 scripts/_build &&
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 -shared -fPIC scripts/pmc_calib.hip -o scripts/_build/libpmc_calib.so &&
export MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_FWD=0 &&
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/gemm_pmc_$1/pmc_fetch -o run -- python3 scripts/prof_act_gemm_pmc.py > gpurun_out/gemm_pmc_$1/fetch.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/gemm_pmc_$1/pmc_write -o run -- python3 scripts/prof_act_gemm_pmc.py > gpurun_out/gemm_pmc_$1/write.log 2>&1
