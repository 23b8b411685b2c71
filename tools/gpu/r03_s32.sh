# Round 3 session 32 (round-end checks): one retrieval partition per CU for the split kernel,
# C3 roofline priced against the split-bf16 ceiling; retrieval tests, C3 bench, filter ablation,
# unblocked bench, kernel stats, then smoke, the whole GPU suite and the default bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_retrieval_gpu.py tests/test_c1_gpu.py -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_s32.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests_s32.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc"; exit $rc; fi
timeout -k 10 300 python -u tools/bench_retrieval.py > gpurun_out/c3_s32.json 2> gpurun_out/c3_s32.err || { echo C3_FAIL; tail -5 gpurun_out/c3_s32.err; exit 1; }
cat gpurun_out/c3_s32.json
TTAMM_RETRIEVAL_ABLATE=1 timeout -k 10 200 python -u tools/bench_retrieval.py --cpu-queries 0 --reps 3 > gpurun_out/c3_s32_ab1.json 2> gpurun_out/c3_s32_ab1.err || { echo AB_FAIL; exit 1; }
timeout -k 10 200 python -u tools/bench_retrieval.py --cpu-queries 0 --reps 3 --blocked 0 > gpurun_out/c3_s32_nob.json 2> gpurun_out/c3_s32_nob.err || { echo NOB_FAIL; tail -5 gpurun_out/c3_s32_nob.err; exit 1; }
for f in ab1 nob; do echo "$f: $(python3 -c "import json;d=json.load(open('gpurun_out/c3_s32_$f.json'));print(d['ms_per_batch'])")"; done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/stats_r -o run -- python3 tools/bench_retrieval.py --cpu-queries 0 > gpurun_out/stats_retr32.json 2> gpurun_out/stats_retr32.err || { echo STATS_FAIL; exit 1; }
find gpurun_out/stats_r -name "*kernel_stats.csv" -exec cp {} gpurun_out/stats_retr32_kernel_stats.csv \;
rm -rf gpurun_out/stats_r
head -4 gpurun_out/stats_retr32_kernel_stats.csv | cut -c1-160
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s32_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/s32_smoke.log; exit 1; }
tail -1 gpurun_out/s32_smoke.log
timeout -k 10 1200 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/s32_gpu_tests.log 2>&1
rc=$?
tail -4 gpurun_out/s32_gpu_tests.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc"; exit $rc; fi
timeout -k 10 600 python -u bench.py > gpurun_out/s32_bench.json 2> gpurun_out/s32_bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/s32_bench.err; exit 1; }
cat gpurun_out/s32_bench.json | cut -c1-400
