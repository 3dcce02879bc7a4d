#!/bin/bash
# full GPU suite + smoke
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ \
  > gpurun_out/r5_full_tests.log 2>&1; rc=$?
tail -15 gpurun_out/r5_full_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5_full_smoke.log 2>&1; rc=$?
tail -3 gpurun_out/r5_full_smoke.log
exit $rc
