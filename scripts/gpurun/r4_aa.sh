#!/bin/bash
# patch conv: residual loads two row segments at a time -- tests, A/B, phase skips
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_convp_gpu.py > gpurun_out/r4_aa_convp_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/prof_convp.py > gpurun_out/r4_aa_convp_ab.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/prof_convp_phases.py > gpurun_out/r4_aa_convp_phases.log 2>&1 || exit 1
