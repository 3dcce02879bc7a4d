# HBM traffic of the physics kernels: FETCH_SIZE and WRITE_SIZE passes (separate runs), calibrated
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/pmc_traffic &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_traffic/pmc_fetch -o run -- python3 scripts/prof_physics.py --calib > gpurun_out/pmc_traffic/fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_traffic/pmc_write -o run -- python3 scripts/prof_physics.py --calib > gpurun_out/pmc_traffic/write.log 2>&1
