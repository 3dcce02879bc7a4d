#!/bin/bash
# narrow phase without per-lane tables: bitwise A/B vs the previous engine, physics time, PMC
# traffic; mipmapped textures: render tests, per-camera cost, frames
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6d
O=gpurun_out/r6d
RMBX_LIB_VARIANT=at-39d4029 timeout -k 10 300 python -u scripts/diag_physics_bitwise.py --out $O/prev.npz > $O/bitwise_prev.log 2>&1 || { tail $O/bitwise_prev.log; exit 1; }
timeout -k 10 300 python -u scripts/diag_physics_bitwise.py --out $O/new.npz --compare $O/prev.npz > $O/bitwise.log 2>&1 || { tail $O/bitwise.log; exit 1; }
cat $O/bitwise.log
rm -f $O/*.npz
for args in "1024" "512" "1024 --env pick"; do
  echo "== prev $args" >> $O/phys_ab.log
  RMBX_LIB_VARIANT=at-39d4029 timeout -k 10 120 python -u scripts/prof_physics.py $args >> $O/phys_ab.log 2>&1 || exit 1
  echo "== new $args" >> $O/phys_ab.log
  timeout -k 10 120 python -u scripts/prof_physics.py $args >> $O/phys_ab.log 2>&1 || exit 1
done
grep -E "==|ms per env-step|per-env front" $O/phys_ab.log
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_fetch -o run -- python3 scripts/prof_physics.py --calib > $O/fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_write -o run -- python3 scripts/prof_physics.py --calib > $O/write.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_render_gpu.py tests/test_render_oracle.py tests/test_env_info_gpu.py tests/test_engine_gpu.py tests/test_pick_gpu.py tests/test_known_answers.py > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed" $O/tests.log | tail -2
grep -E "^FAILED|^ERROR|textured pixels" $O/tests.log | head -12
[ $rc -le 1 ] || exit $rc
OUT=$O timeout -k 10 300 python -u scripts/prof_render_materials.py > $O/render_materials.log 2>&1 || { tail -20 $O/render_materials.log; exit 1; }
cat $O/render_materials.log
exit $rc
