#!/bin/bash
# closed-loop parity test, Pick qacc bar, divergence curves of the engine vs the oracle
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -v -s --timeout 400 --timeout-method thread tests/test_closed_loop_gpu.py tests/test_pick_gpu.py > gpurun_out/r6_a_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r6_a_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u scripts/diag_divergence.py --out gpurun_out/r6_divergence > gpurun_out/r6_a_div.log 2>&1 || { tail -20 gpurun_out/r6_a_div.log; exit 1; }
cat gpurun_out/r6_a_div.log
