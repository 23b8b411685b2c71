# Round 4, session 1: smoke, the step parity tests (incl. the ragged full/short/full batches),
# the self-launching 2-rank bench, the default C2 bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s1_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/s1_smoke.log; exit 1; }
tail -1 gpurun_out/s1_smoke.log
timeout -k 10 900 python -u -m pytest tests/test_step_parity_gpu.py tests/test_sharded_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/s1_tests.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/s1_tests.log; exit 1; }
tail -3 gpurun_out/s1_tests.log
timeout -k 10 600 python -u bench.py > gpurun_out/s1_bench.json 2> gpurun_out/s1_bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/s1_bench.err; exit 1; }
cat gpurun_out/s1_bench.json
