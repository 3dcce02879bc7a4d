#!/bin/bash
# the whole GPU suite (no bench)
# usage: bash scripts/gpurun/r6_full.sh <tag>
set -o pipefail
T=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/${T}_gpu_tests.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/${T}_gpu_tests.log | tail -3
grep -E "^FAILED|^ERROR" gpurun_out/${T}_gpu_tests.log | head -20
exit $rc
