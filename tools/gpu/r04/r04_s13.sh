# Round 4, session 13: the aux-stream difference — the slice alone overlapping the backward GEMMs
# (prologue forked after the MLP, slice on the aux stream); the replay without packed math
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
DIAG_MODE=repeat TTAMM_DIAG_JOIN=2 timeout -k 10 300 python -u tools/diag/deferred_c2.py > gpurun_out/s13_j2_sliceaux.txt 2>&1; echo "join 2, slice on aux"; grep -E " w:|Error|error" gpurun_out/s13_j2_sliceaux.txt | tail -n 4
DIAG_MODE=repeat TTAMM_REPLAY_NOPK=1 timeout -k 10 300 python -u tools/diag/deferred_c2.py > gpurun_out/s13_nopk.txt 2>&1; echo "no packed math"; grep -E " w:|Error|error" gpurun_out/s13_nopk.txt | tail -n 4
DIAG_MODE=repeat TTAMM_REPLAY_SCALAR=1 timeout -k 10 300 python -u tools/diag/deferred_c2.py > gpurun_out/s13_scalar.txt 2>&1; echo "scalar-constant replay"; grep -E " w:|Error|error" gpurun_out/s13_scalar.txt | tail -n 4
