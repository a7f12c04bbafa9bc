# Parity tests, then a C2 and a C3 bench line (no CPU baseline).  usage: scripts/gpu_quick.sh TAG
TAG=${1:-q}
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
DINO_SYNC_CHECK=1 scripts/gpu_step.sh 300 gpurun_out/${TAG}_e4.log -- python scripts/exp_batches.py 512 full 0,0,512 && \
scripts/gpu_step.sh 600 gpurun_out/${TAG}_tests.log -- python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread && \
scripts/gpu_step.sh 300 gpurun_out/${TAG}_c2.log -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline && \
scripts/gpu_step.sh 300 gpurun_out/${TAG}_c3.log -- python bench.py --mixed --images 4096 --unique 128 --steps 8 --warmup 2 --no-cpu-baseline
