set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_round5.py -x -q -p no:cacheprovider --timeout 300 > gpurun_out/r5_t5.log 2>&1; rc=$?
tail -4 gpurun_out/r5_t5.log; exit $rc
