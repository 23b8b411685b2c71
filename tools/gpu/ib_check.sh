# in-batch parity tests, then the C4 / C2 in-batch bench lines (developer script)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_inbatch_gpu.py tests/test_sharded_gpu.py -x -q --timeout 120 --timeout-method thread -k "inbatch or in_batch" > gpurun_out/ib_tests.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --config c4 > gpurun_out/b_c4.json 2> gpurun_out/b_c4.err
TTAMM_IB_ONE_BLOCK=1 timeout -k 10 300 python bench.py --no-cpu-baseline --config c4 > gpurun_out/b_c4_one.json 2> gpurun_out/b_c4_one.err
timeout -k 10 300 python bench.py --no-cpu-baseline --negatives in-batch > gpurun_out/b_c2ib.json 2> gpurun_out/b_c2ib.err
