set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6ls
DINO_INGEST_LIB=build/lib_lsmall.so timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_round6.py -k "lane or damaged" > gpurun_out/r6ls/tests.log 2>&1 || { tail -20 gpurun_out/r6ls/tests.log; exit 1; }
tail -1 gpurun_out/r6ls/tests.log
R6TAG=r6ls bash scripts/gpu_prog_ab.sh wave:X=1 lane:DINO_PROG_LANE=1 lsmall:DINO_INGEST_LIB=build/lib_lsmall.so,DINO_PROG_LANE=1 lsmall_e4:DINO_INGEST_LIB=build/lib_lsmall.so,DINO_PROG_LANE=1,DINO_SIDE_ENGINES=4,DINO_SIDE_MAX=256 lsmall_m1024:DINO_INGEST_LIB=build/lib_lsmall.so,DINO_PROG_LANE=1,DINO_SIDE_MAX=1024
