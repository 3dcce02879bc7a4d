#!/bin/bash
# front-kernel LDS layout (collision scratch in the dead cinert / crb region): physics A/B vs the
# commit before, bitwise state comparison, engine tests
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for v in at-HEAD "" at-HEAD ""; do
  echo "== variant '$v' cable" >> gpurun_out/r5_y_front_lds_ab.log
  RMBX_LIB_VARIANT=$v timeout -k 10 200 python -u scripts/prof_physics.py >> gpurun_out/r5_y_front_lds_ab.log 2>&1 || exit 1
done
for v in at-HEAD ""; do
  echo "== variant '$v' pick" >> gpurun_out/r5_y_front_lds_ab.log
  RMBX_LIB_VARIANT=$v timeout -k 10 200 python -u scripts/prof_physics.py 1024 --env pick >> gpurun_out/r5_y_front_lds_ab.log 2>&1 || exit 1
done
for v in at-HEAD ""; do
  RMBX_LIB_VARIANT=$v timeout -k 10 200 python -u scripts/phys_state_dump.py >> gpurun_out/r5_y_front_lds_ab.log 2>&1 || exit 1
  RMBX_LIB_VARIANT=$v timeout -k 10 200 python -u scripts/phys_state_dump.py --env pick >> gpurun_out/r5_y_front_lds_ab.log 2>&1 || exit 1
done
python -c "
import numpy as np
for s in ('cable','pick'):
    a=np.load(f'gpurun_out/phys_state_at-HEAD_{s}.npy'); b=np.load(f'gpurun_out/phys_state_default_{s}.npy')
    print(s, 'bitwise equal:', np.array_equal(a,b), 'max diff', float(np.abs(a-b).max()))
" >> gpurun_out/r5_y_front_lds_ab.log 2>&1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_engine_gpu.py tests/test_insert_gpu.py > gpurun_out/r5_y_engine_tests.log 2>&1 || { tail -30 gpurun_out/r5_y_engine_tests.log; exit 1; }
tail -2 gpurun_out/r5_y_engine_tests.log
