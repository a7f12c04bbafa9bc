# One GPU session: sync-checked full batch, parity tests, bench, rocprof stats.
# usage: scripts/gpu_round.sh TAG
TAG=${1:-run}
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 && \
DINO_SYNC_CHECK=1 scripts/gpu_step.sh 300 gpurun_out/${TAG}_e4.log -- python scripts/exp_batches.py 512 full 0,0,512 && \
scripts/gpu_step.sh 600 gpurun_out/${TAG}_tests.log -- python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread && \
scripts/gpu_step.sh 900 gpurun_out/${TAG}_bench.log -- python bench.py --steps 20 --warmup 3 --h2d --e2e --kernel-json gpurun_out/${TAG}_kernels.json && \
scripts/gpu_step.sh 900 gpurun_out/${TAG}_prof.log -- rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --images 8192 --procs 0 --depth 1
