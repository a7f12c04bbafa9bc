cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
for d in 1 2 3 4; do timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --depth $d > gpurun_out/depth_$d.log 2>&1 || exit 1; done
