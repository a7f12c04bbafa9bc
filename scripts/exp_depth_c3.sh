cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
for d in 2 3 4 6; do timeout -k 10 300 python bench.py --mixed --images 4096 --unique 128 --steps 8 --warmup 2 --no-cpu-baseline --depth $d > gpurun_out/dc3_$d.log 2>&1 || exit 1; done
