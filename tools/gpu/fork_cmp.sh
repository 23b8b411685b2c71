set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu-baseline --config c5 > gpurun_out/fk_late.json 2> gpurun_out/fk.err
TTAMM_EARLY_FORK=1 timeout -k 10 300 python bench.py --no-cpu-baseline --config c5 > gpurun_out/fk_early.json 2> gpurun_out/fk.err
timeout -k 10 300 python bench.py --no-cpu-baseline --config c5 > gpurun_out/fk_late2.json 2> gpurun_out/fk.err
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_step_parity_gpu.py -k bf16 > gpurun_out/fk_tests.log 2>&1
