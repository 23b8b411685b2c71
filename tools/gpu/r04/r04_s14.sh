# Round 4, session 14: the fast replay with pair-layout constants (no broadcast operands in its
# packed loop), full overlap: run-to-run and against the eager sweep
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
DIAG_MODE=repeat timeout -k 10 300 python -u tools/diag/deferred_c2.py > gpurun_out/s14_repeat.txt 2>&1; echo "pairs, repeat"; grep -E " w:| m:|Error|error" gpurun_out/s14_repeat.txt | tail -n 8
DIAG_MODE=overlap timeout -k 10 300 python -u tools/diag/deferred_c2.py > gpurun_out/s14_overlap.txt 2>&1; grep -E " w:|Error|error" gpurun_out/s14_overlap.txt | tail -n 4
timeout -k 10 300 python -u -m pytest tests/test_deferred_gpu.py -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/s14_deferred.log 2>&1; tail -n 2 gpurun_out/s14_deferred.log
timeout -k 10 120 ./two-tower-augmented-with-adaptive-mimic-mechanism_amd/build/replay_bench > gpurun_out/s14_replay_bench.txt 2>&1; tail -n 6 gpurun_out/s14_replay_bench.txt
