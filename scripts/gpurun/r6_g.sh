#!/bin/bash
# renderer register budget with textures: 8 (default) / 6 / 5 waves per SIMD
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6g
O=gpurun_out/r6g
for v in default render6 render5; do
  echo "== $v" >> $O/render_waves.log
  if [ $v = default ]; then unset RMBX_LIB_VARIANT; else export RMBX_LIB_VARIANT=$v; fi
  OUT=$O timeout -k 10 300 python -u scripts/prof_render_materials.py >> $O/render_waves.log 2>&1 || { tail -20 $O/render_waves.log; exit 1; }
done
grep -E "==|front|side" $O/render_waves.log
