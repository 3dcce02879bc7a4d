# fp32 ACT pieces, then DP graph capture at the batch sizes the cap excluded
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out &&
MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_FWD=0 timeout -k 10 900 python -u scripts/prof_act_fp32.py --batch 1024 --benchmark 1 > gpurun_out/r2_prof_act_fp32_v2.log 2>&1 &&
for cfg in "1024 fp32" "256 bf16" "1024 bf16"; do
  set -- $cfg
  timeout -k 10 300 python -u scripts/diag_dp_capture.py $1 $2 > gpurun_out/r2_dp_capture_$1_$2.log 2>&1; rc=$?
  echo "diag rc=$rc" >> gpurun_out/r2_dp_capture_$1_$2.log
  [ $rc -lt 124 ] || exit $rc
done
