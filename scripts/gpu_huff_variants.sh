# Huffman work-item shape sweep (lanes per item x stream bits per item): C2 and C3 bench lines.
TAG=${1:-hv}
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
for k in ${VARIANTS:-t128s512 t256s1024 t128s768}; do \
  DINO_INGEST_LIB=build/lib_$k.so DINO_SYNC_CHECK=1 scripts/gpu_step.sh 300 gpurun_out/${TAG}_chk_$k.log -- python scripts/exp_batches.py 512 full 0,0,512 && \
  DINO_INGEST_LIB=build/lib_$k.so scripts/gpu_step.sh 300 gpurun_out/${TAG}_c2_$k.log -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline && \
  DINO_INGEST_LIB=build/lib_$k.so scripts/gpu_step.sh 300 gpurun_out/${TAG}_c3_$k.log -- python bench.py --mixed --images 4096 --unique 128 --steps 8 --warmup 2 --no-cpu-baseline || exit 1; \
done
