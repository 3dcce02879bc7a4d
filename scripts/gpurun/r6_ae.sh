#!/bin/bash
# round-6: patch conv with the past-the-image waves skipping their MFMAs -- tests, A/B (interleaved)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6ae
O=gpurun_out/r6ae
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_convp_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
: > $O/ab.log
for r in 1 2; do
  RMBX_CONVP_DEAD=1 timeout -k 10 300 python -u scripts/prof_convp_ab.py >> $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
  RMBX_CONVP_DEAD=0 timeout -k 10 300 python -u scripts/prof_convp_ab.py >> $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
done
grep -v amdgpu.ids $O/ab.log
