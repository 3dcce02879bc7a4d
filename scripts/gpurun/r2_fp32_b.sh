cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out &&
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_nn_gpu.py -k "f32 or s2d" tests/test_act_full_gpu.py tests/test_bad_state_gpu.py > gpurun_out/r2_tests_b.log 2>&1 &&
MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_FWD=0 timeout -k 10 600 python -u scripts/prof_act_fp32.py --batch 1024 --benchmark 1 > gpurun_out/r2_prof_act_fp32_v3.log 2>&1 &&
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --no_cpu_baseline > gpurun_out/r2_bench_probe.json 2> gpurun_out/r2_bench_probe.err &&
{ MIOPEN_ENABLE_LOGGING=1 MIOPEN_LOG_LEVEL=5 AMD_LOG_LEVEL=1 timeout -k 10 300 python -u scripts/diag_dp_capture.py 1024 fp32 --steps 2 > gpurun_out/r2_dp_capture_1024_fp32_log.log 2>&1; echo "diag rc=$?" >> gpurun_out/r2_dp_capture_1024_fp32_log.log; }
