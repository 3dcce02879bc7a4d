#!/bin/bash
# round 3: F(4x4) Winograd: kernel tests + per-layer timing, ACT production-config parity with it,
# then the default bench with F(2x2) and with F(4x4)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_winograd_gpu.py -k winograd4 > gpurun_out/r3_wino4_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/prof_winograd4.py 1024 --dbg > gpurun_out/r3_wino4_prof.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -ne 0 ] && exit $rc
RMBX_WINO_TILE=f4 timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_act_full_gpu.py > gpurun_out/r3_act_full_f4.log 2>&1
rc=$?; echo "act f4 rc=$rc"; [ $rc -ne 0 ] && exit $rc
RMBX_WINO_TILE=f4 timeout -k 10 400 python bench.py --no_cpu_baseline > gpurun_out/r3_bench_f4.json.log 2> gpurun_out/r3_bench_f4.err
rc=$?; echo "bench f4 rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --no_cpu_baseline > gpurun_out/r3_bench_f2.json.log 2> gpurun_out/r3_bench_f2.err
echo "bench f2 rc=$?"
