#!/bin/bash
# round 4 records: the full GPU suite, smoke, the default bench (CPU baseline + bf16 secondary), the
# bench under rocprofv3 (timed-window summary), the f16x3 GEMM HBM-traffic PMC passes
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r4_final_gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_final_smoke.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/r4_final_bench.json.log 2> gpurun_out/r4_final_bench.err || exit 1
bash scripts/gpurun/r3_benchprof.sh r4final || exit 1
bash scripts/gpurun/gemm_pmc.sh r4final || exit 1
timeout -k 10 200 python -u scripts/prof_stem_phases.py > gpurun_out/r4_final_stem_phases.log 2>&1 || exit 1
