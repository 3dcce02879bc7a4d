#!/bin/bash
# records after the front-kernel LDS layout: full GPU suite, smoke, default + driver-shaped bench,
# physics PMC traffic
set -o pipefail
T=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/${T}_gpu_tests.log 2>&1 || { tail -30 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -2 gpurun_out/${T}_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1 || { tail -20 gpurun_out/${T}_smoke.log; exit 1; }
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench.json.log 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench_driver_shape.json.log 2> gpurun_out/${T}_bench_driver_shape.err || { tail -20 gpurun_out/${T}_bench_driver_shape.err; exit 1; }
bash scripts/gpurun/pmc_traffic.sh || exit 1
echo records done
