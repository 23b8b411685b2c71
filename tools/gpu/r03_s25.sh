# Round 3 session 25: retrieval with the compaction check as one ballot per wave (tests + C3
# bench), then SQ counters of the C3 retrieval kernel (what bounds retrieval_x_kernel)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_retrieval_gpu.py tests/test_c1_gpu.py -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_s25.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests_s25.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc"; exit $rc; fi
timeout -k 10 300 python -u tools/bench_retrieval.py > gpurun_out/c3_s25.json 2> gpurun_out/c3_s25.err || { echo C3_FAIL; tail -5 gpurun_out/c3_s25.err; exit 1; }
cat gpurun_out/c3_s25.json
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/pmc_retr -o run -- python3 tools/bench_retrieval.py --queries 16384 > gpurun_out/pmc_retr.txt 2>&1 || { echo PMC_FAIL; tail -5 gpurun_out/pmc_retr.txt; exit 1; }
find gpurun_out/pmc_retr -name "*counter_collection.csv" -exec cp {} gpurun_out/pmc_retr_sq.csv \;
rm -rf gpurun_out/pmc_retr
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmc_retr2 -o run -- python3 tools/bench_retrieval.py --queries 16384 > gpurun_out/pmc_retr2.txt 2>&1 || { echo PMC2_FAIL; tail -5 gpurun_out/pmc_retr2.txt; exit 1; }
find gpurun_out/pmc_retr2 -name "*counter_collection.csv" -exec cp {} gpurun_out/pmc_retr_sq2.csv \;
rm -rf gpurun_out/pmc_retr2
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/stats_r -o run -- python3 tools/bench_retrieval.py > gpurun_out/stats_retr.json 2> gpurun_out/stats_retr.err || { echo STATS_FAIL; exit 1; }
find gpurun_out/stats_r -name "*kernel_stats.csv" -exec cp {} gpurun_out/stats_retr_kernel_stats.csv \;
rm -rf gpurun_out/stats_r
head -5 gpurun_out/stats_retr_kernel_stats.csv | cut -c1-160
