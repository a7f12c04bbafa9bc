# wave-decoder fix check + the exit-time SIGSEGV hunt: the same rocprofv3
# command three times, every process writing its library map at exit
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r6k
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_round6.py -k damaged tests/test_gpu_round2.py::test_progressive_and_raw_decode_bit_exact tests/test_gpu_round2.py::test_writer_multiscan_cases_through_k_prog tests/test_gpu_round2.py::test_damaged_streams_through_the_abi > $OUT/tests.log 2>&1; echo "tests rc $?"; tail -8 $OUT/tests.log
for rep in 1 2 3; do
  mkdir -p $OUT/maps$rep
  DINO_EXIT_MAPS=$OUT/maps$rep/{pid}.txt timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof$rep -o run --output-format csv -- python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-extras > $OUT/prof$rep.log 2>&1
  rc=$?
  echo "prof $rep rc $rc"
  if [ $rc -ne 0 ]; then grep -n "SIGSEGV\|Aborted\|PC:\|@ \|dumped" $OUT/prof$rep.log | head -30; exit 0; fi
done
