# round-6 lane decoder session: progressive parity tests, per-scan phases (lane / wave),
# decode capacity, and the c2_prog leg
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${R6TAG:-r6b}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_round6.py tests/test_gpu_round2.py::test_progressive_and_raw_decode_bit_exact tests/test_gpu_round2.py::test_writer_multiscan_cases_through_k_prog tests/test_gpu_round2.py::test_damaged_streams_through_the_abi tests/test_gpu_round3.py::test_side_route_matches_in_batch_device_route > $OUT/tests.log 2>&1 || echo TESTS FAILED
tail -9 $OUT/tests.log
DINO_PROG_LANE=1 timeout -k 10 120 python -u scripts/prog_phases.py 2>&1 | grep -v amdgpu.ids > $OUT/phases_lane.txt
timeout -k 10 120 python -u scripts/prog_phases.py 2>&1 | grep -v amdgpu.ids > $OUT/phases_wave.txt
cat $OUT/phases_lane.txt $OUT/phases_wave.txt
timeout -k 10 200 python -u scripts/prog_scale.py --ns 64,512,1024,2048 --reps 3 --streams 4 2>&1 | grep case > $OUT/prog_scale.jsonl
cat $OUT/prog_scale.jsonl
DINO_SIDE_TIMING=1 timeout -k 10 300 python -u bench.py --only-leg c2_prog --steps 96 --warmup 5 > $OUT/prog.json 2> $OUT/prog.err
tail -c 1200 $OUT/prog.json
