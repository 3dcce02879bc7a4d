#!/bin/bash
# round 3: DP / DP3 production-size parity, then kernel traces of the config-4/5 workloads
set -o pipefail
mkdir -p gpurun_out
export MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_FWD=0
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 500 --timeout-method thread -m gpu tests/test_policy_parity_gpu.py > gpurun_out/r3_policy_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r3_prof_dp -o dp -- python3 scripts/bench_policy.py DiffusionPolicy --num_envs 2048 --precision bf16 --steps 24 --warmup 24 > gpurun_out/r3_prof_dp.log 2>&1
rc=$?; echo "prof dp rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r3_prof_dp3 -o dp3 -- python3 scripts/bench_policy.py DiffusionPolicy3d --num_envs 1024 --tactile --precision fp32 --steps 24 --warmup 24 > gpurun_out/r3_prof_dp3.log 2>&1
echo "prof dp3 rc=$?"
find gpurun_out -name "*_kernel_trace.csv" -delete
find gpurun_out -name "*.db" -delete
du -sh gpurun_out
