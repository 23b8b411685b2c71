# Round 3 session 7: retrieval with the per-tile max pre-check (tests, C3 bench split / fp32, one
# SQ counter pass), default bench kernel stats with the rewritten score kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_retrieval_gpu.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_s7.log 2>&1
rc=$?
tail -5 gpurun_out/gpu_tests_s7.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc"; exit $rc; fi
timeout -k 10 300 python -u tools/bench_retrieval.py > gpurun_out/c3_split.json 2> gpurun_out/c3_split.err || { echo C3_FAIL; tail -5 gpurun_out/c3_split.err; exit 1; }
cat gpurun_out/c3_split.json
TTAMM_RETRIEVAL_FP32=1 timeout -k 10 300 python -u tools/bench_retrieval.py > gpurun_out/c3_fp32.json 2> gpurun_out/c3_fp32.err || { echo C3F_FAIL; exit 1; }
cat gpurun_out/c3_fp32.json
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/pmc_retr -o run -- python3 tools/bench_retrieval.py --queries 16384 > gpurun_out/pmc_retr.txt 2>&1 || { echo PMC_FAIL; tail -5 gpurun_out/pmc_retr.txt; exit 1; }
find gpurun_out/pmc_retr -name "*counter_collection.csv" -exec cp {} gpurun_out/pmc_retr_sq.csv \;
rm -rf gpurun_out/pmc_retr
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/stats -o run -- python3 bench.py --no-cpu-baseline > gpurun_out/stats_bench.json 2> gpurun_out/stats.err || { echo STATS_FAIL; exit 1; }
find gpurun_out/stats -name "*kernel_stats.csv" -exec cp {} gpurun_out/stats_kernel_stats.csv \;
rm -rf gpurun_out/stats

export TMPDIR=/tmp
for c in 0 32 64 128; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --aux-cus $c > gpurun_out/b_aux$c.json 2> gpurun_out/b_aux$c.err || { echo AUX${c}_FAIL; tail -5 gpurun_out/b_aux$c.err; exit 1; }
done
python3 -c "
import json
for c in (0,32,64,128):
    d=json.load(open('gpurun_out/b_aux%d.json'%c)); r=d['roofline']
    print(c, d['value'], d['ms_per_step'], r['ms_per_step'], r.get('parts_ms_per_step'), [(k['kernel'][:20], k.get('avg_launch_ms')) for k in d['kernels'][1:]])
"
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/pmc_step -o run -- python3 bench.py --no-cpu-baseline --steps 40 --warmup 3 > gpurun_out/pmc_step.txt 2>&1 || { echo PMC_FAIL; tail -5 gpurun_out/pmc_step.txt; exit 1; }
find gpurun_out/pmc_step -name "*counter_collection.csv" -exec cp {} gpurun_out/pmc_step_sq.csv \;
rm -rf gpurun_out/pmc_step
echo done
