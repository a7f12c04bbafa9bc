# Timing runs of library variants: C2 and C3 bench lines per variant.
# VARIANTS="lib[:ENV=VAL[,ENV=VAL]] ..." (build/lib_<lib>.so, optional environment)
TAG=${1:-kn}
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
for v in ${VARIANTS:-base}; do \
  k=${v%%:*}; e=""; [ "$k" != "$v" ] && e=${v#*:}; n=$(echo "$v" | tr ':=,' '___'); \
  env ${e//,/ } DINO_INGEST_LIB=build/lib_$k.so scripts/gpu_step.sh 300 gpurun_out/${TAG}_c2_$n.log -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline && \
  env ${e//,/ } DINO_INGEST_LIB=build/lib_$k.so scripts/gpu_step.sh 300 gpurun_out/${TAG}_c3_$n.log -- python bench.py --mixed --images 4096 --unique 128 --steps 8 --warmup 2 --no-cpu-baseline || exit 1; \
done
