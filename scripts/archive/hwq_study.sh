set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
for q in 4 8; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --only-leg e2e --procs 16 > gpurun_out/hwq_e2e_$q.json 2> gpurun_out/hwq_e2e_$q.err || exit $?
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-extras > gpurun_out/hwq_c2_$q.json 2> gpurun_out/hwq_c2_$q.err || exit $?
done
for q in 4 8; do head -c 300 gpurun_out/hwq_e2e_$q.json; echo; python scripts/show_bench.py gpurun_out/hwq_c2_$q.json; done
