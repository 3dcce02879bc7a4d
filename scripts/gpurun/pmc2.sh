# physics PMC: calibrated HBM traffic (FETCH_SIZE / WRITE_SIZE passes), SQ stall counters, icache
# usage: bash scripts/gpurun/pmc2.sh <tag>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/pmc_$1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_$1/pmc_fetch -o run -- python3 scripts/prof_physics.py --calib > gpurun_out/pmc_$1/fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_$1/pmc_write -o run -- python3 scripts/prof_physics.py --calib > gpurun_out/pmc_$1/write.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_IFETCH SQ_INSTS --kernel-include-regex "front|solver" -d gpurun_out/pmc_$1/sq -o run --output-format csv -- python3 scripts/phys_one.py > gpurun_out/pmc_$1/sq.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE --kernel-include-regex "front|solver" -d gpurun_out/pmc_$1/ic -o run --output-format csv -- python3 scripts/phys_one.py > gpurun_out/pmc_$1/ic.log 2>&1
