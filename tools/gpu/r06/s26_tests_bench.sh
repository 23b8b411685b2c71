# full GPU suite + smoke + the driver's bench command on the device-scope-event tree
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s26_gpu_tests.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s26_smoke.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/s26_bench.json 2> gpurun_out/s26_bench.err
