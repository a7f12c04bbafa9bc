# C3 (mixed resolution + iBOT masks) and C5-dtype (fp8 epilogue) bench lines.
# usage: scripts/gpu_configs.sh TAG
TAG=${1:-cfg}
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
scripts/gpu_step.sh 600 gpurun_out/${TAG}_c3.log -- python bench.py --mixed --images 8192 --steps 10 --warmup 2 --no-cpu-baseline --h2d && \
scripts/gpu_step.sh 600 gpurun_out/${TAG}_fp8.log -- python bench.py --dtype fp8 --steps 20 --warmup 3 --no-cpu-baseline --e2e
