#!/bin/bash
# round 3: Winograd F(4x4) with the per-channel-count schedule defaults: tests, HBM traffic passes,
# then the default bench (no CPU leg)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_winograd_gpu.py > gpurun_out/r3_wf_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
bash scripts/gpurun/wino_pmc.sh $1 f4 || { echo "pmc failed"; exit 1; }
echo "pmc ok"
timeout -k 10 600 python -u bench.py --no_cpu_baseline > gpurun_out/r3_wf_bench_$1.json.log 2> gpurun_out/r3_wf_bench_$1.err
rc=$?; echo "bench rc=$rc"; tail -c 3000 gpurun_out/r3_wf_bench_$1.json.log; exit $rc
