# round 2 first GPU pass: new parity tests, fp32 bench probe, DP graph-capture diagnostic (last)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out &&
true &&
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no_cpu_baseline > gpurun_out/r2_bench_fp32_probe.log 2>&1 &&
{ MIOPEN_ENABLE_LOGGING=1 MIOPEN_LOG_LEVEL=5 timeout -k 10 300 python scripts/diag_dp_capture.py 256 fp32 > gpurun_out/r2_dp_capture_256_fp32.log 2>&1; rc=$?; echo "diag rc=$rc" >> gpurun_out/r2_dp_capture_256_fp32.log; [ $rc -lt 124 ]; }
