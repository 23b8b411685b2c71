# the shipped binary after the last rebuild: smoke, the core parity tests and the driver's bench command
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s43_smoke.log 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "step_parity or deferred or fullsize or c1 or index_errors" > gpurun_out/s43_tests.log 2>&1
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/s43_driver.json 2> gpurun_out/s43_driver.err
