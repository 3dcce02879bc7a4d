#!/bin/bash
# round-6: render tests + bench with the round-filling render groups
set -o pipefail
T=r6ad
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6ad
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_render_gpu.py tests/test_multicam_gpu.py tests/test_shard_gpu.py > gpurun_out/r6ad/tests.log 2>&1 || { tail -30 gpurun_out/r6ad/tests.log; exit 1; }
tail -2 gpurun_out/r6ad/tests.log
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 --no_cpu_baseline --no_bf16_secondary > gpurun_out/${T}_bench.json.log 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/${T}_bench.json.log').read().strip().splitlines()[-1])
print('value', d['value'], 'ms', d['ms_per_step'], 'phases', d.get('phases',{}).get('ms_per_env_step'))
c=d.get('c3_per_rank'); print('c3', c and (c['value'], c['phases']['ms_per_env_step']))
"
