#!/bin/bash
# small-grid GEMMs on the 128 / 64-wide tile: C4 (DiffusionPolicy x2048 fp32) and C5 with the commit
# before (at-HEAD) and with the change, plus the GEMM tests
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
L=gpurun_out/r5_y5_gemm_fill_ab.log
for v in at-HEAD ""; do
  echo "== variant '$v'" >> $L
  RMBX_LIB_VARIANT=$v timeout -k 10 400 python scripts/bench_policy.py DiffusionPolicy --num_envs 2048 --precision fp32 2>&1 | tail -1 >> $L || exit 1
done
for v in at-HEAD ""; do
  echo "== variant '$v'" >> $L
  RMBX_LIB_VARIANT=$v timeout -k 10 400 python scripts/bench_policy.py DiffusionPolicy --num_envs 2048 --precision fp32 2>&1 | tail -1 >> $L || exit 1
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gemm_gpu.py tests/test_policy_parity_gpu.py tests/test_act_batch_gpu.py > gpurun_out/r5_y5_tests.log 2>&1 || { tail -30 gpurun_out/r5_y5_tests.log; exit 1; }
tail -2 gpurun_out/r5_y5_tests.log
