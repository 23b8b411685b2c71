# Round 3 session 5: coalesce bit-exact + sharded L_cal tests first, then the whole GPU suite,
# then the default bench and its kernel-trace --stats summary.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_coalesce_gpu.py tests/test_sharded_options_gpu.py -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_new.log 2>&1
rc=$?
tail -30 gpurun_out/gpu_tests_new.log
if [ $rc -ne 0 ]; then echo "new tests rc=$rc"; exit $rc; fi
timeout -k 10 1700 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 900 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -15 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
timeout -k 10 600 python -u bench.py > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || { echo BENCH_FAIL; tail -20 gpurun_out/bench_c2.err; exit 1; }
cat gpurun_out/bench_c2.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/stats -o run -- python3 bench.py --no-cpu-baseline > gpurun_out/stats_bench.json 2> gpurun_out/stats.err || { echo STATS_FAIL; exit 1; }
find gpurun_out/stats -name "*kernel_stats.csv" -exec cp {} gpurun_out/stats_kernel_stats.csv \;
rm -rf gpurun_out/stats
echo "pytest rc=$rc"
