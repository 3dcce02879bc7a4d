#!/bin/bash
# contact diagnostic of the Newton-test states + render-with-meshes timing
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/diag_contacts.py > gpurun_out/r5_c_contacts.log 2>&1 || { echo "diag rc=$?"; tail -20 gpurun_out/r5_c_contacts.log; exit 1; }
timeout -k 10 300 python -u scripts/prof_render_mesh.py > gpurun_out/r5_c_render.log 2>&1 || { echo "render rc=$?"; tail -20 gpurun_out/r5_c_render.log; exit 1; }
cat gpurun_out/r5_c_render.log
