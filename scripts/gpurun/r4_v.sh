#!/bin/bash
# patch-staged convs in the backbone: ACT parity tests, then the bench A/B (patch on / off)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_act_full_gpu.py tests/test_act_batch_gpu.py tests/test_convp_gpu.py tests/test_policy_parity_gpu.py tests/test_multicam_gpu.py tests/test_nn_gpu.py > gpurun_out/r4_v_act_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --no_cpu_baseline --no_bf16_secondary > gpurun_out/r4_v_bench_patch.json.log 2> gpurun_out/r4_v_bench_patch.err || exit 1
RMBX_S1_PATCH= timeout -k 10 400 python -u bench.py --no_cpu_baseline --no_bf16_secondary > gpurun_out/r4_v_bench_nopatch.json.log 2> gpurun_out/r4_v_bench_nopatch.err || exit 1
