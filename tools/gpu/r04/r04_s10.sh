# Round 4, session 10: is the fast deferred replay's run-to-run difference a stream race or the
# kernel?  (overlap on / off; scalar-constant replay; no packed math)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
DIAG_MODE=overlap timeout -k 10 300 python -u tools/diag/deferred_c2.py > gpurun_out/s10_overlap.txt 2>&1; grep -v amdgpu.ids gpurun_out/s10_overlap.txt | grep -E " w:| m:|Error|error" | tail -n 12
DIAG_MODE=scalar TTAMM_REPLAY_SCALAR=1 timeout -k 10 300 python -u tools/diag/deferred_c2.py > gpurun_out/s10_scalar.txt 2>&1; grep -v amdgpu.ids gpurun_out/s10_scalar.txt | grep -E " w:| m:|Error|error" | tail -n 6
DIAG_MODE=scalar TTAMM_REPLAY_NOPK=1 timeout -k 10 300 python -u tools/diag/deferred_c2.py > gpurun_out/s10_nopk.txt 2>&1; grep -v amdgpu.ids gpurun_out/s10_nopk.txt | grep -E " w:| m:|Error|error" | tail -n 6
