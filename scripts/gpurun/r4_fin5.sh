#!/bin/bash
# round-4 records after the net-change Hessian (solver without spills, physics traffic 3.08 GB): the GPU
# suite, smoke, bench (CPU leg), bench
# under rocprofv3 (timed window), the GEMM HBM-traffic PMC passes
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r4_fin5_gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_fin5_smoke.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/r4_fin5_bench.json.log 2> gpurun_out/r4_fin5_bench.err || exit 1
bash scripts/gpurun/r3_benchprof.sh r4fin5 || exit 1
bash scripts/gpurun/gemm_pmc.sh r4fin5 || exit 1
