#!/bin/bash
# texture cost split at 6 waves per SIMD (RMBX_RENDER_DBG 512: no footprint, 128: base level, 256: no sampling)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6h
O=gpurun_out/r6h
for dbg in 0 512 128 256; do
  echo "== RMBX_RENDER_DBG=$dbg" >> $O/render_split.log
  RMBX_RENDER_DBG=$dbg OUT=$O timeout -k 10 300 python -u scripts/prof_render_materials.py >> $O/render_split.log 2>&1 || { tail -20 $O/render_split.log; exit 1; }
done
grep -E "==|front" $O/render_split.log
