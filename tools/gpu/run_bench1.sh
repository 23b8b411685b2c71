set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_inbatch_gpu.py tests/test_sharded_gpu.py tests/test_index_errors_gpu.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/t2.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b_c2_sampled.json 2> gpurun_out/b_c2_sampled.err
timeout -k 10 300 python bench.py --no-cpu-baseline --negatives in-batch > gpurun_out/b_c2_ib.json 2> gpurun_out/b_c2_ib.err
timeout -k 10 300 python bench.py --no-cpu-baseline --negatives in-batch --neg 5 > gpurun_out/b_c2_ib5.json 2> gpurun_out/b_c2_ib5.err
timeout -k 10 400 python bench.py --no-cpu-baseline --config c4 > gpurun_out/b_c4.json 2> gpurun_out/b_c4.err
