cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out &&
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_bad_state_gpu.py tests/test_known_answers.py tests/test_engine_gpu.py tests/test_product_schedule.py tests/test_checkpoint.py tests/test_pick_gpu.py > gpurun_out/r2_tests_c.log 2>&1 &&
for cfg in "1024 fp32" "1024 bf16" "2048 fp32" "2048 bf16"; do
  set -- $cfg
  timeout -k 10 300 python -X faulthandler -u scripts/diag_dp_capture.py $1 $2 > gpurun_out/r2_dp_capture_gemm_$1_$2.log 2>&1; rc=$?
  echo "diag rc=$rc" >> gpurun_out/r2_dp_capture_gemm_$1_$2.log
  [ $rc -eq 0 ] || exit $rc
done
