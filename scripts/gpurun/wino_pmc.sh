# HBM traffic of the Winograd f32 conv: FETCH_SIZE and WRITE_SIZE passes (separate runs)
# usage: bash scripts/gpurun/wino_pmc.sh <tag> [f4|f2]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/wino_pmc_$1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/wino_pmc_$1/pmc_fetch -o run -- python3 scripts/prof_winograd_pmc.py --tile ${2:-f4} > gpurun_out/wino_pmc_$1/fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/wino_pmc_$1/pmc_write -o run -- python3 scripts/prof_winograd_pmc.py --tile ${2:-f4} > gpurun_out/wino_pmc_$1/write.log 2>&1
