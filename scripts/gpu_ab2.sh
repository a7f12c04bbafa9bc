cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_round2.py -q -m gpu -k "extreme or damaged or golden" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ab2_tests.log 2>&1; tail -2 gpurun_out/ab2_tests.log; \
bash scripts/gpu_ab.sh ab2 a b c
