#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python3 -u scripts/proto_bf16x6.py > gpurun_out/proto6.log 2>&1 && \
timeout -k 10 400 python3 -u bench.py --no_cpu_baseline > gpurun_out/bench_base.json.log 2> gpurun_out/bench_base.err
