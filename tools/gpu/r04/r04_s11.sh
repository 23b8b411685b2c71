# Round 4, session 11: which part of the aux-stream overlap makes the fast deferred replay differ
# run to run: the rolling slice on the aux stream (TTAMM_SLICE_MAIN=1 moves it to the main stream)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
DIAG_MODE=repeat timeout -k 10 300 python -u tools/diag/deferred_c2.py > gpurun_out/s11_base.txt 2>&1; grep -E " w:|Error|error" gpurun_out/s11_base.txt | tail -n 6
DIAG_MODE=repeat TTAMM_SLICE_MAIN=1 timeout -k 10 300 python -u tools/diag/deferred_c2.py > gpurun_out/s11_slicemain.txt 2>&1; grep -E " w:|Error|error" gpurun_out/s11_slicemain.txt | tail -n 6
DIAG_MODE=repeat TTAMM_SLICE_LATE=1 timeout -k 10 300 python -u tools/diag/deferred_c2.py > gpurun_out/s11_slicelate.txt 2>&1; grep -E " w:|Error|error" gpurun_out/s11_slicelate.txt | tail -n 6
