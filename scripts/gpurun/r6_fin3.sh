#!/bin/bash
# round-6 final records: full GPU suite + smoke, driver-shaped bench, the bench under rocprofv3 --kernel-trace --stats
set -o pipefail
T=r6fin3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/${T}
timeout -k 10 1000 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/${T}_gpu_tests.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/${T}_gpu_tests.log | tail -2
grep -E "^FAILED|^ERROR" gpurun_out/${T}_gpu_tests.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1 || { tail -20 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench.json.log 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/${T}_bench.json.log').read().strip().splitlines()[-1])
print('value', d['value'], 'ms', d['ms_per_step'], 'phases', d.get('phases',{}).get('ms_per_env_step'))
c=d.get('c3_per_rank'); print('c3', c and (c['value'], c['ms_per_step'], c['physics_kernel_ms'], c['phases']['ms_per_env_step']))
print('roofline', d['roofline']['frac'], 'conv', d['roofline_conv3x3']['frac'], 'bf16', d.get('secondary_bf16',{}).get('value'), 'cpu', d.get('cpu_baseline',{}).get('value'))
"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}/prof -o run -- python3 bench.py --no_cpu_baseline --no_bf16_secondary --no_c3_per_rank --steps 20 --warmup 5 > gpurun_out/${T}/bench_under_rocprof.json.log 2> gpurun_out/${T}/prof.err || { tail -20 gpurun_out/${T}/prof.err; exit 1; }
find gpurun_out/${T} -name "*_kernel_trace.csv" -size +40M -delete
echo done
timeout -k 10 300 python -u scripts/prof_render_cams.py > gpurun_out/${T}_render_cams.log 2>&1 || { tail -20 gpurun_out/${T}_render_cams.log; exit 1; }
grep -v amdgpu.ids gpurun_out/${T}_render_cams.log
