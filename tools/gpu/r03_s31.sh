# Round 3 session 31: retrieval partitions for the split kernel sized for one block per CU
# (C3: 6 -> 1 partition); retrieval tests, C3 bench, partition sweep 1/2/3/6
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_retrieval_gpu.py tests/test_c1_gpu.py -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_s31.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests_s31.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc"; exit $rc; fi
timeout -k 10 300 python -u tools/bench_retrieval.py > gpurun_out/c3_s31.json 2> gpurun_out/c3_s31.err || { echo C3_FAIL; tail -5 gpurun_out/c3_s31.err; exit 1; }
cat gpurun_out/c3_s31.json
for p in 2 3 6; do
  TTAMM_RETRIEVAL_PARTS=$p timeout -k 10 200 python -u tools/bench_retrieval.py --cpu-queries 0 --reps 3 > gpurun_out/c3_s31_p$p.json 2> gpurun_out/c3_s31_p$p.err || { echo P_FAIL $p; exit 1; }
  echo "parts $p: $(python3 -c "import json;d=json.load(open('gpurun_out/c3_s31_p$p.json'));print(d['ms_per_batch'])")"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/stats_r -o run -- python3 tools/bench_retrieval.py --cpu-queries 0 > gpurun_out/stats_retr31.json 2> gpurun_out/stats_retr31.err || { echo STATS_FAIL; exit 1; }
find gpurun_out/stats_r -name "*kernel_stats.csv" -exec cp {} gpurun_out/stats_retr31_kernel_stats.csv \;
rm -rf gpurun_out/stats_r
head -4 gpurun_out/stats_retr31_kernel_stats.csv | cut -c1-160
