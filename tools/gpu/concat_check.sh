set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_step_parity_gpu.py tests/test_kernels_gpu.py tests/test_golden_gpu.py tests/test_sharded_gpu.py > gpurun_out/concat.log 2>&1
