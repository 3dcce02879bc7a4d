#!/bin/bash
# round-6: driver-shaped bench with the render cache
set -o pipefail
T=r6u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench.json.log 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/${T}_bench.json.log').read().strip().splitlines()[-1])
print('value', d['value'], 'ms', d['ms_per_step'], 'phases', d.get('phases',{}).get('ms_per_env_step'))
c=d.get('c3_per_rank'); print('c3', c and (c['value'], c['ms_per_step'], c['physics_kernel_ms'], c['phases']['ms_per_env_step']))
print('roofline', d['roofline']['frac'], 'conv', d['roofline_conv3x3']['frac'], 'bf16', d.get('secondary_bf16',{}).get('value'), 'cpu', d.get('cpu_baseline',{}).get('value'))
"
