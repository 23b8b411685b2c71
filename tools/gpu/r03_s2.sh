# C2 full-size parity details + the rest of the GPU suite from test_step_parity on
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_fullsize_parity_gpu.py -k c2 -x -p no:cacheprovider --timeout 600 --timeout-method thread -rA --tb=long > gpurun_out/c2_full.log 2>&1
echo "c2 rc=$?"
grep -E "Error|assert|rel err" gpurun_out/c2_full.log | head -20
timeout -k 10 900 python -u -m pytest tests/test_step_parity_gpu.py tests/test_retrieval_gpu.py tests/test_route_gpu.py -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests2.log 2>&1
rc=$?
tail -15 gpurun_out/gpu_tests2.log
echo "pytest rc=$rc"
