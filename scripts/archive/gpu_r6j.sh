set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6j
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_round6.py > gpurun_out/r6j/tests.log 2>&1; echo "tests rc $?"
tail -12 gpurun_out/r6j/tests.log
DINO_EXIT_MAPS=gpurun_out/r6j/maps.txt timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6j/prof -o run --output-format csv -- python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-extras > gpurun_out/r6j/prof.log 2>&1; echo "prof rc $?"
grep -n "SIGSEGV\|Aborted\|PC:\|@ " gpurun_out/r6j/prof.log | head -30
