#!/bin/bash
# render: parity of the default build, then RASTER_SMALL A/B (per-camera call time)
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
bash scripts/gpurun/r5_i.sh || exit 1
for v in rsmall2 rsmall4 rsmall16 rsmall32; do
  RMBX_LIB_VARIANT=$v RENDER_ONLY_ASSET=1 RENDER_ALL_CAMS=1 timeout -k 10 200 python -u scripts/prof_render_mesh.py > gpurun_out/r5_l_$v.log 2>&1 || { echo "$v rc=$?"; exit 1; }
  echo "== $v"; grep "ms per" gpurun_out/r5_l_$v.log
done
