set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_step_parity_gpu.py -m gpu -q -k bf16 --timeout 200 --timeout-method thread > gpurun_out/tb.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --config c5 > gpurun_out/b_c5.json 2> gpurun_out/b_c5.err
