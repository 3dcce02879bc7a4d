#!/bin/bash
# round-6: back-face culling in the visibility pass -- render tests (oracle culls too), then the cache A/B
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6w
O=gpurun_out/r6w
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_render_gpu.py tests/test_multicam_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -u scripts/prof_render_cache.py > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log
