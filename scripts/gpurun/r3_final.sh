#!/bin/bash
# round 3 end-of-round measurement on one tree: full GPU suite, smoke, the default bench (CPU leg
# included), then the bench under rocprofv3 (kernel stats + timed window)
# usage: bash scripts/gpurun/r3_final.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/full_tests_$1.log 2>&1
rc=$?
tail -3 gpurun_out/full_tests_$1.log
if [ $rc -ne 0 ] && ! grep -q " passed" gpurun_out/full_tests_$1.log; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$1.log 2>&1 &&
timeout -k 10 600 python -u bench.py > gpurun_out/bench_$1.json.log 2> gpurun_out/bench_$1.err &&
bash scripts/gpurun/r3_benchprof.sh $1
rc2=$?
exit $(( rc != 0 ? rc : rc2 ))
