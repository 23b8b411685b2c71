set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu-baseline --config c4 > gpurun_out/b_c4.json 2> gpurun_out/b_c4.err
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_fullsize_gpu.py > gpurun_out/fullsize.log 2>&1
