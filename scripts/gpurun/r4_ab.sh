#!/bin/bash
# ACT forward without the one-camera cat copy and with mem + pos from the last LayerNorm pass:
# ACT parity tests, then the bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_act_full_gpu.py tests/test_act_batch_gpu.py tests/test_policy_parity_gpu.py tests/test_multicam_gpu.py tests/test_rollout_gpu.py > gpurun_out/r4_ab_act_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --no_cpu_baseline --no_bf16_secondary > gpurun_out/r4_ab_bench.json.log 2> gpurun_out/r4_ab_bench.err || exit 1
