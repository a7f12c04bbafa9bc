# Experiment: k_huff3 with its sparse-entry / block-info / DC stores compiled out
# (timing only; outputs invalid), plus SQ counters of the default build.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
DINO_INGEST_LIB=build/lib_nostore.so timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --images 8192 > gpurun_out/ns_c2.log 2>&1; \
DINO_INGEST_LIB=build/lib_nostore.so timeout -k 10 300 python bench.py --mixed --images 4096 --unique 128 --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/ns_c3.log 2>&1; \
BENCH="python bench.py --steps 2 --warmup 1 --no-cpu-baseline --images 2048 --unique 64 --procs 0 --depth 1" && \
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d gpurun_out/sq2_a -o run --output-format csv -- $BENCH > gpurun_out/sq2_a.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_BRANCH -d gpurun_out/sq2_b -o run --output-format csv -- $BENCH > gpurun_out/sq2_b.log 2>&1 ; \
python scripts/pmc_counters.py gpurun_out/sq2_a gpurun_out/sq2_b > gpurun_out/sq2_table.txt 2>&1
