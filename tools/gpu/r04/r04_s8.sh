# Round 4, session 8: the two bitwise tests that failed in s7 (deferred = eager at C2, C1 epoch
# device loader vs host batches), with and without the 128x96 wide-output tiles
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="tests/test_deferred_gpu.py::test_deferred_c2_equals_eager tests/test_data_gpu.py::test_c1_epoch_from_binary_files_matches_host_batches"
timeout -k 10 300 python -u -m pytest $T -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/s8_a.log 2>&1; tail -n 3 gpurun_out/s8_a.log
TTAMM_GEMM_WIDE_TILES=1 timeout -k 10 300 python -u -m pytest $T -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/s8_b.log 2>&1; tail -n 3 gpurun_out/s8_b.log
timeout -k 10 300 python -u -m pytest tests/test_deferred_gpu.py -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/s8_c.log 2>&1; tail -n 5 gpurun_out/s8_c.log
echo done
