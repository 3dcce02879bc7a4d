#!/bin/bash
# round-6: fma_mix split remainders -- parity tests, A/B, phase skips
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6aa
O=gpurun_out/r6aa
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_attention_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 200 python -u scripts/prof_attn_dma.py > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log
timeout -k 10 200 python -u scripts/prof_attn_phases.py > $O/phases.log 2>&1 || { tail -20 $O/phases.log; exit 1; }
cat $O/phases.log
