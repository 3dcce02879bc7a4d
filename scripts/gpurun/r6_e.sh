#!/bin/bash
# mip sampling speed-up: render tests + per-camera cost
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6e
O=gpurun_out/r6e
timeout -k 10 400 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_render_gpu.py tests/test_env_info_gpu.py > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed" $O/tests.log | tail -2
grep -E "^FAILED|^ERROR|textured pixels" $O/tests.log | head -12
[ $rc -le 1 ] || exit $rc
OUT=$O timeout -k 10 300 python -u scripts/prof_render_materials.py > $O/render_materials.log 2>&1 || { tail -20 $O/render_materials.log; exit 1; }
cat $O/render_materials.log
exit $rc
