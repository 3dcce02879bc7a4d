#!/bin/bash
# textured renderer: render / oracle tests, env info, closed loop, multicam; per-camera cost; bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_render_gpu.py tests/test_render_oracle.py tests/test_env_info_gpu.py tests/test_closed_loop_gpu.py tests/test_multicam_gpu.py > gpurun_out/r6c_tests.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/r6c_tests.log | tail -2
grep -E "^FAILED|^ERROR|textured pixels" gpurun_out/r6c_tests.log | head -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u scripts/prof_render_materials.py > gpurun_out/r6c_render_materials.log 2>&1 || { tail -20 gpurun_out/r6c_render_materials.log; exit 1; }
cat gpurun_out/r6c_render_materials.log
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6c_bench.json.log 2> gpurun_out/r6c_bench.err || { tail -20 gpurun_out/r6c_bench.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/r6c_bench.json.log').read().strip().splitlines()[-1])
print('value', d['value'], 'ms', d['ms_per_step'], 'phases', d.get('phases',{}).get('ms_per_env_step'))
c=d.get('c3_per_rank'); print('c3', c and (c['value'], c['ms_per_step'], c['physics_kernel_ms'], c['phases']['ms_per_env_step']))
print('roofline', d['roofline']['frac'], 'bf16', d.get('secondary_bf16',{}).get('value'), 'cpu', d.get('cpu_baseline',{}).get('value'))
"
exit $rc
