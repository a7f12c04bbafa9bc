# HBM traffic per kernel launch: two PMC passes (FETCH_SIZE, WRITE_SIZE) of the same
# short bench command (serialised batches, 8192 images, > L3) for one workload.
# usage: scripts/gpu_pmc.sh TAG [extra bench args]   (e.g. TAG=c3 --mixed; TAG=fp8 --dtype fp8)
TAG=${1:-pmc}
shift
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
BENCH="python bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-extras --images 8192 --procs 0 --depth 1 $*" && \
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${TAG}_fetch -o run --output-format csv -- $BENCH > gpurun_out/${TAG}_fetch.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${TAG}_write -o run --output-format csv -- $BENCH > gpurun_out/${TAG}_write.log 2>&1 && \
python scripts/pmc_traffic.py gpurun_out/${TAG}_fetch gpurun_out/${TAG}_write gpurun_out/${TAG}_traffic.json
