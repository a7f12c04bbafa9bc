cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 200 python scripts/huff_phases.py > gpurun_out/ph_async.txt 2>&1 && \
DINO_PHASE_LIB=build/lib_phases_rounds.so timeout -k 10 200 python scripts/huff_phases.py > gpurun_out/ph_rounds.txt 2>&1 && \
timeout -k 10 200 python scripts/huff_phases.py --mixed > gpurun_out/ph_async_m.txt 2>&1 && \
DINO_PHASE_LIB=build/lib_phases_rounds.so timeout -k 10 200 python scripts/huff_phases.py --mixed > gpurun_out/ph_rounds_m.txt 2>&1
for f in gpurun_out/ph_*.txt; do echo "== $f"; tail -6 $f; done
