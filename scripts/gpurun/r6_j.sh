#!/bin/bash
# round-6 counter records: GEMM / patch-conv HBM traffic (FETCH / WRITE), MFMA utilisation
# (SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE) over one fp32 ACT inference, and the default bench
# under rocprofv3 --kernel-trace --stats
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6j scripts/_build
O=gpurun_out/r6j
export MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_FWD=0
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 -shared -fPIC scripts/pmc_calib.hip -o scripts/_build/libpmc_calib.so || exit 1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_fetch -o run -- python3 scripts/prof_act_gemm_pmc.py > $O/fetch.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_write -o run -- python3 scripts/prof_act_gemm_pmc.py > $O/write.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA --kernel-trace --output-format csv -d $O/sq -o run -- python3 scripts/prof_act_gemm_pmc.py > $O/sq.log 2>&1 || exit 1
python3 scripts/mfma_util.py $(find $O/sq -name "*counter_collection.csv" | head -1) > $O/mfma_util.txt || exit 1
cat $O/mfma_util.txt | head -20
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no_cpu_baseline --steps 20 --warmup 5 > $O/bench_under_rocprof.json.log 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
find $O -name "*_kernel_trace.csv" -size +20M -delete
echo done
