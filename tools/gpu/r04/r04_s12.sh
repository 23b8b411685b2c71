# Round 4, session 12: the aux-stream race, bisected by forcing joins (TTAMM_DIAG_JOIN=1: the
# grouping joined before the backward; =2: the prologue forked after the feature MLP)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for j in 1 2; do
DIAG_MODE=repeat TTAMM_SLICE_MAIN=1 TTAMM_DIAG_JOIN=$j timeout -k 10 300 python -u tools/diag/deferred_c2.py > gpurun_out/s12_j$j.txt 2>&1; echo "join $j"; grep -E " w:|Error|error" gpurun_out/s12_j$j.txt | tail -n 4
done
