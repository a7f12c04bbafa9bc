# Huffman segment-size sweep: GPU parity tests with the default build, then C2 and C3
# bench lines per variant (default lib + build/lib_seg*.so).
TAG=${1:-seg}
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
DINO_SYNC_CHECK=1 scripts/gpu_step.sh 300 gpurun_out/${TAG}_e4.log -- python scripts/exp_batches.py 512 full 0,0,512 && \
scripts/gpu_step.sh 600 gpurun_out/${TAG}_tests.log -- python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread && \
for k in ${VARIANTS:-default 1024 4096}; do \
  if [ $k = default ]; then L=dataloader_amd/libdino_ingest.so; else L=build/lib_seg$k.so; fi; \
  DINO_INGEST_LIB=$L scripts/gpu_step.sh 300 gpurun_out/${TAG}_c2_$k.log -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline || exit 1; \
  DINO_INGEST_LIB=$L scripts/gpu_step.sh 300 gpurun_out/${TAG}_c3_$k.log -- python bench.py --mixed --images 4096 --unique 128 --steps 8 --warmup 2 --no-cpu-baseline || exit 1; \
done
