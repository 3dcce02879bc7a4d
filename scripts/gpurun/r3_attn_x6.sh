#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_attention_gpu.py > gpurun_out/attn_x6_tests.log 2>&1 || exit 1
timeout -k 10 200 python3 -u scripts/prof_attention_f32.py > gpurun_out/prof_attn_x6.log 2>&1 || exit 1
timeout -k 10 500 python3 -u -m pytest -x -v -s --timeout 480 --timeout-method thread tests/test_act_full_gpu.py > gpurun_out/act_full_attnx6.log 2>&1 || exit 1
timeout -k 10 500 python3 -u bench.py --no_cpu_baseline > gpurun_out/bench_attnx6.json.log 2> gpurun_out/bench_attnx6.err
