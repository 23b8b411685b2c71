set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -q --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_deferred_gpu.py > gpurun_out/ab_deferred.log 2>&1 || true
TTAMM_SLICE_MAIN=1 timeout -k 10 300 $T tests/test_c1_gpu.py -k losses > gpurun_out/ab_c1_main.log 2>&1 || true
timeout -k 10 300 $T tests/test_c1_gpu.py -k losses > gpurun_out/ab_c1_aux.log 2>&1 || true
