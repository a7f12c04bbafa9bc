cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
DINO_SYNC_CHECK=1 scripts/gpu_step.sh 300 gpurun_out/e1.log -- python scripts/exp_batches.py 512 decode 0,0,0 && \
DINO_SYNC_CHECK=1 scripts/gpu_step.sh 300 gpurun_out/e4.log -- python scripts/exp_batches.py 512 full 0,0,512 && \
scripts/gpu_step.sh 600 gpurun_out/t3.log -- python -m pytest tests/test_gpu_parity.py -q -m gpu && \
scripts/gpu_step.sh 900 gpurun_out/bench1.log -- python bench.py --steps 20 --warmup 3 --h2d --kernel-json gpurun_out/kernels1.json && \
scripts/gpu_step.sh 900 gpurun_out/prof1.log -- rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --images 8192
