cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
scripts/gpu_step.sh 300 gpurun_out/dbg.log -- python scripts/gpu_debug_decode.py && \
scripts/gpu_step.sh 900 gpurun_out/t1.log -- python -m pytest tests/test_gpu_parity.py -q -m gpu && \
scripts/gpu_step.sh 300 gpurun_out/smoke1.log -- python -c "import __graft_entry__ as g; g.smoke()"
