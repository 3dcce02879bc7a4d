#!/bin/bash
# render determinism + per-camera render time + kernel split
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpurun/r5_full.sh || exit 1

RENDER_ONLY_ASSET=1 RENDER_ALL_CAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5_h_prof -o r5h --output-format csv -- \
  python3 -u scripts/prof_render_mesh.py > gpurun_out/r5_h_render.log 2>&1 || { echo "prof rc=$?"; tail -20 gpurun_out/r5_h_render.log; exit 1; }
cat gpurun_out/r5_h_render.log | grep -v "^\[\|W2" | tail -8
f=$(ls gpurun_out/r5_h_prof/*/r5h_kernel_stats.csv 2>/dev/null | head -1 || true)
[ -n "$f" ] && grep -i "raster\|render_kernel" "$f" | cut -c1-220
exit 0
