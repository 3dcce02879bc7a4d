#!/bin/bash
# compact collision scratch (7-double geom records + type bytes, 16-bit survivor pair indices): Pick
# 45.1 -> 38.8 KiB per env (four envs per CU) vs the commit before; physics, bitwise states, tests
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
L=gpurun_out/r5_y4_collision_compact_ab.log
for v in at-HEAD "" at-HEAD ""; do
  echo "== variant '$v' pick 2048" >> $L
  RMBX_LIB_VARIANT=$v timeout -k 10 200 python -u scripts/prof_physics.py 2048 --env pick >> $L 2>&1 || exit 1
done
for v in at-HEAD ""; do
  echo "== variant '$v' pick 1024" >> $L
  RMBX_LIB_VARIANT=$v timeout -k 10 200 python -u scripts/prof_physics.py 1024 --env pick >> $L 2>&1 || exit 1
  echo "== variant '$v' cable 1024" >> $L
  RMBX_LIB_VARIANT=$v timeout -k 10 200 python -u scripts/prof_physics.py >> $L 2>&1 || exit 1
done
rm -f gpurun_out/phys_state_*.npy
for v in at-HEAD ""; do
  RMBX_LIB_VARIANT=$v timeout -k 10 200 python -u scripts/phys_state_dump.py >> $L 2>&1 || exit 1
  RMBX_LIB_VARIANT=$v timeout -k 10 200 python -u scripts/phys_state_dump.py --env pick >> $L 2>&1 || exit 1
done
python -c "
import numpy as np
for s in ('cable','pick'):
    a=np.load(f'gpurun_out/phys_state_at-HEAD_{s}.npy'); b=np.load(f'gpurun_out/phys_state_default_{s}.npy')
    print(s, 'bitwise equal:', np.array_equal(a,b), 'max diff', float(np.abs(a-b).max()))
" >> $L 2>&1
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_engine_gpu.py tests/test_insert_gpu.py tests/test_pick_workloads_gpu.py tests/test_pick_gpu.py tests/test_front_lds_gpu.py > gpurun_out/r5_y4_tests.log 2>&1 || { tail -30 gpurun_out/r5_y4_tests.log; exit 1; }
tail -2 gpurun_out/r5_y4_tests.log
