cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
DINO_SYNC_CHECK=1 scripts/gpu_step.sh 600 gpurun_out/bench0.log -- python bench.py --steps 3 --warmup 1 --images 2048 --no-cpu-baseline && \
scripts/gpu_step.sh 900 gpurun_out/bench1.log -- python bench.py --steps 20 --warmup 3 --h2d --kernel-json gpurun_out/kernels1.json && \
scripts/gpu_step.sh 900 gpurun_out/prof1.log -- rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --images 8192
