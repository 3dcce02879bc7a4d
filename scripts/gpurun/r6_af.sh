#!/bin/bash
# round-6: render per-pixel loads a tile ahead -- render tests, then the ray-cast pass under rocprofv3
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6af
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_render_gpu.py tests/test_multicam_gpu.py > gpurun_out/r6af/tests.log 2>&1 || { tail -30 gpurun_out/r6af/tests.log; exit 1; }
tail -2 gpurun_out/r6af/tests.log
for n in a b; do
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6af/$n -o run -- python3 scripts/prof_raster_probe.py > gpurun_out/r6af/$n.log 2>&1 || { tail -5 gpurun_out/r6af/$n.log; exit 1; }
find gpurun_out/r6af/$n -name "*_kernel_trace.csv" -delete
python3 -c "
import csv,glob
f=glob.glob('gpurun_out/r6af/$n/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'render_kernel' in r['Name'] or 'raster' in r['Name']: print('$n', r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')
"
done
