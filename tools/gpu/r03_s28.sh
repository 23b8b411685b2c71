# Round 3 session 28: retrieval with per-query counts and thresholds in registers and ballot-ordered
# candidate slots (no LDS atomics): tests, C3 bench, the filter ablation and the unblocked bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_retrieval_gpu.py tests/test_c1_gpu.py -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_s28.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests_s28.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc"; exit $rc; fi
timeout -k 10 300 python -u tools/bench_retrieval.py > gpurun_out/c3_s28.json 2> gpurun_out/c3_s28.err || { echo C3_FAIL; tail -5 gpurun_out/c3_s28.err; exit 1; }
cat gpurun_out/c3_s28.json
TTAMM_RETRIEVAL_ABLATE=1 timeout -k 10 200 python -u tools/bench_retrieval.py --cpu-queries 0 --reps 3 > gpurun_out/c3_s28_ab1.json 2> gpurun_out/c3_s28_ab1.err || { echo AB_FAIL; exit 1; }
timeout -k 10 200 python -u tools/bench_retrieval.py --cpu-queries 0 --reps 3 --blocked 0 > gpurun_out/c3_s28_nob.json 2> gpurun_out/c3_s28_nob.err || { echo NOB_FAIL; exit 1; }
for f in ab1 nob; do echo "$f: $(python3 -c "import json;d=json.load(open('gpurun_out/c3_s28_$f.json'));print(d['ms_per_batch'])")"; done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/stats_r -o run -- python3 tools/bench_retrieval.py --cpu-queries 0 > gpurun_out/stats_retr28.json 2> gpurun_out/stats_retr28.err || { echo STATS_FAIL; exit 1; }
find gpurun_out/stats_r -name "*kernel_stats.csv" -exec cp {} gpurun_out/stats_retr28_kernel_stats.csv \;
rm -rf gpurun_out/stats_r
head -4 gpurun_out/stats_retr28_kernel_stats.csv | cut -c1-160
