# Round 3 session 10 (re-entry): whole GPU suite on the rebuilt HEAD, smoke, default bench with the
# CPU baseline, kernel stats of the default bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1500 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/gpu_tests_s10.log 2>&1
rc=$?
tail -15 gpurun_out/gpu_tests_s10.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_s10.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/smoke_s10.log; exit 1; }
cat gpurun_out/smoke_s10.log
timeout -k 10 600 python -u bench.py > gpurun_out/bench_s10.json 2> gpurun_out/bench_s10.err || { echo BENCH_FAIL; tail -20 gpurun_out/bench_s10.err; exit 1; }
cat gpurun_out/bench_s10.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/stats -o run -- python3 bench.py --no-cpu-baseline > gpurun_out/stats_bench_s10.json 2> gpurun_out/stats_s10.err || { echo STATS_FAIL; exit 1; }
find gpurun_out/stats -name "*kernel_stats.csv" -exec cp {} gpurun_out/stats_kernel_stats_s10.csv \;
rm -rf gpurun_out/stats
echo "pytest rc=$rc"
