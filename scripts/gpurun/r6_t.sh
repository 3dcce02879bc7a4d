#!/bin/bash
# round-6: static-background render cache -- render tests, then the A/B
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6t
O=gpurun_out/r6t
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_render_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -u scripts/prof_render_cache.py > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log
