# Round 4, session 46: 512 blocks per role kept for sharded in-batch (Bc > 2B) — the in-batch and
# sharded tests, the emulated 8-rank C4 line and C4
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_inbatch_gpu.py tests/test_inbatch_op_gpu.py tests/test_sharded_gpu.py tests/test_sharded_options_gpu.py > gpurun_out/s46_tests.log 2>&1 || { echo TESTS_FAIL; tail -20 gpurun_out/s46_tests.log; exit 1; }
tail -n 1 gpurun_out/s46_tests.log
timeout -k 10 500 python -u bench.py --no-cpu-baseline --emulate-world 8 --config c4 --steps 30 --warmup 3 > gpurun_out/s46_c4_emu8.json 2> gpurun_out/s46_c4_emu8.err || { echo BENCH_FAIL; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/s46_c4_emu8.json')); print('c4_emu8', d['value'], d['ms_per_step'])"
timeout -k 10 400 python -u bench.py --no-cpu-baseline --config c4 > gpurun_out/s46_c4.json 2> gpurun_out/s46_c4.err || { echo BENCH_FAIL; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/s46_c4.json')); print('c4', d['value'], d['ms_per_step'])"
