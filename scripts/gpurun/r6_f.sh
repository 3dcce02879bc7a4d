#!/bin/bash
# texture sampling cost split (RMBX_RENDER_DBG 128: base level only, 256: no sampling)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6f
O=gpurun_out/r6f
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_render_gpu.py > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for dbg in 0 128 256; do
  echo "== RMBX_RENDER_DBG=$dbg" >> $O/render_split.log
  RMBX_RENDER_DBG=$dbg OUT=$O timeout -k 10 300 python -u scripts/prof_render_materials.py >> $O/render_split.log 2>&1 || { tail -20 $O/render_split.log; exit 1; }
done
grep -E "==|front" $O/render_split.log
