# Huffman variants (prebuilt into build/): phase profiles.  default = 256 lanes, no LDS window.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
DINO_HUFF_PROFILE=1 scripts/gpu_step.sh 300 gpurun_out/h256_g.log -- python scripts/exp_huff.py 512 && \
DINO_HUFF_PROFILE=1 DINO_INGEST_LIB=build/lib_h512_g.so scripts/gpu_step.sh 300 gpurun_out/h512_g.log -- python scripts/exp_huff.py 512 && \
DINO_HUFF_PROFILE=1 DINO_INGEST_LIB=build/lib_h256_w.so scripts/gpu_step.sh 300 gpurun_out/h256_w.log -- python scripts/exp_huff.py 512
