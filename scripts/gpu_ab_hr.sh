set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
bash scripts/gpu_ab.sh abhr_c2 pf0 pf4 pf8 pf0 pf4 > gpurun_out/abhr_c2.txt 2>&1 || exit $?
AB_ARGS="--mixed --no-extras --images 4096 --unique 512 --steps 20" bash scripts/gpu_ab.sh abhr_c3 pf0 pf4 pf8 pf0 pf4 > gpurun_out/abhr_c3.txt 2>&1 || exit $?
