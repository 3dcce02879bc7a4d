#!/bin/bash
# round-6: cached render-kernel probes (groups per env, phase skips) under rocprofv3
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6ac
run() {  # name, env...
  n=$1; shift
  env "$@" timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6ac/$n -o run -- python3 scripts/prof_raster_probe.py > gpurun_out/r6ac/$n.log 2>&1 || { tail -5 gpurun_out/r6ac/$n.log; exit 1; }
  find gpurun_out/r6ac/$n -name "*_kernel_trace.csv" -delete
  python3 -c "
import csv,glob
f=glob.glob('gpurun_out/r6ac/$n/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'render_kernel<true' in r['Name'] and '2>' not in r['Name']: print('$n', r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')
"
}
run g4 RMBX_RENDER_GROUPS=4
run g6 RMBX_RENDER_GROUPS=6
run g8 RMBX_RENDER_GROUPS=8
run g12 RMBX_RENDER_GROUPS=12
run g16 RMBX_RENDER_GROUPS=16
run nc8 RMBX_RENDER_GROUPS=8 RMBX_RENDER_CACHE=0
run nc16 RMBX_RENDER_GROUPS=16 RMBX_RENDER_CACHE=0
