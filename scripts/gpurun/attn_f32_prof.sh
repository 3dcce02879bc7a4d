# f32 attention: parity tests + profile
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out &&
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_attention_gpu.py -k f32 > gpurun_out/attn_tests_$1.log 2>&1 &&
timeout -k 10 200 python scripts/prof_attention_f32.py 1024 > gpurun_out/attn_f32_prof_$1.log 2>&1
