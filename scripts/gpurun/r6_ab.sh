#!/bin/bash
# round-6: raster pass phase probes under rocprofv3
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6ab
for d in 0 16 32 64; do
  RMBX_RENDER_DBG=$d timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6ab/d$d -o run -- python3 scripts/prof_raster_probe.py > gpurun_out/r6ab/d$d.log 2>&1 || { tail -5 gpurun_out/r6ab/d$d.log; exit 1; }
  find gpurun_out/r6ab/d$d -name "*_kernel_trace.csv" -delete
  python3 -c "
import csv,glob
f=glob.glob('gpurun_out/r6ab/d$d/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'raster' in r['Name'] or 'render_kernel' in r['Name']: print('dbg $d', r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')
"
done
