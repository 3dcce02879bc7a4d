#!/bin/bash
# driver-shaped bench (steps 20 / warmup 5) with the pre-split GEMMs, A/B against RMBX_GEMM_PRESPLIT=0
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no_bf16_secondary --no_cpu_baseline \
  > gpurun_out/r5_n_bench.json.log 2> gpurun_out/r5_n_bench.err || { echo "bench rc=$?"; tail -20 gpurun_out/r5_n_bench.err; exit 1; }
RMBX_GEMM_PRESPLIT=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no_bf16_secondary --no_cpu_baseline \
  > gpurun_out/r5_n_bench_nops.json.log 2> gpurun_out/r5_n_bench_nops.err || { echo "bench rc=$?"; tail -20 gpurun_out/r5_n_bench_nops.err; exit 1; }
for f in gpurun_out/r5_n_bench.json.log gpurun_out/r5_n_bench_nops.json.log; do
python -c "import json,sys;d=json.load(open('$f'));r=d['roofline'];print('$f',d['value'],d['ms_per_step'],d['policy_inference_us_per_call'],r['frac'],r['ms_per_inference']);print(json.dumps(d.get('phases',{}).get('ms_per_env_step')))"
done
