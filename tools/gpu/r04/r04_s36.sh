# Round 4, session 36: (1) narrow (128x96) 32-k bf16 tiles on two register sets, (2) GEMM
# epilogues that request a 4-row chunk's operands before its stores.  Parity (step, bf16,
# full-size), then C2 and C5 (default tiles, every bf16 GEMM narrow, wgrads narrow too)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_step_parity_gpu.py tests/test_fullsize_parity_gpu.py > gpurun_out/s36_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/s36_tests.log; exit 1; }
tail -2 gpurun_out/s36_tests.log
for cfg in "" "--config c4"; do
  timeout -k 10 400 python -u bench.py --no-cpu-baseline $cfg > gpurun_out/s36_x.json 2> gpurun_out/s36_x.err || { echo BENCH_FAIL; tail -5 gpurun_out/s36_x.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/s36_x.json')); print('[$cfg]', d['value'], d['ms_per_step'])"
done
for pre in "" "TTAMM_GEMM_NARROW_BF16=1" "TTAMM_GEMM_NARROW_BF16=1 TTAMM_WGRAD_ALL_NARROW=1" ""; do
  env $pre timeout -k 10 400 python -u bench.py --no-cpu-baseline --config c5 > gpurun_out/s36_x.json 2> gpurun_out/s36_x.err || { echo BENCH_FAIL; tail -5 gpurun_out/s36_x.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/s36_x.json')); print('c5 [$pre]', d['value'], d['ms_per_step'])"
done
