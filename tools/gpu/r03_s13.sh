# Round 3 session 13: vectorised score kernel (parity tests + bench), VALU issue rates, SQ counters
# of the default bench, steady-state kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
B=two-tower-augmented-with-adaptive-mimic-mechanism_amd/build
timeout -k 10 900 python -u -m pytest tests/test_step_parity_gpu.py tests/test_inbatch_gpu.py tests/test_sharded_gpu.py tests/test_sharded_options_gpu.py tests/test_golden_gpu.py tests/test_category_gpu.py -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_s13.log 2>&1
rc=$?
tail -15 gpurun_out/gpu_tests_s13.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc"; exit $rc; fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/b_s13.json 2> gpurun_out/b_s13.err || { echo B_FAIL; tail -5 gpurun_out/b_s13.err; exit 1; }
python3 -c "
import json
d=json.load(open('gpurun_out/b_s13.json')); print(d['value'], d['ms_per_step'], d['final_loss'])"
timeout -k 10 120 $B/valu_bench > gpurun_out/valu_bench.txt 2>&1 || { echo VB_FAIL; cat gpurun_out/valu_bench.txt; exit 1; }
cat gpurun_out/valu_bench.txt
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/pmc_step -o run -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/pmc_step.txt 2>&1 || { echo PMC_FAIL; tail -5 gpurun_out/pmc_step.txt; exit 1; }
find gpurun_out/pmc_step -name "*counter_collection.csv" -exec cp {} gpurun_out/pmc_step_sq.csv \;
rm -rf gpurun_out/pmc_step
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_l -o run -- python3 bench.py --no-cpu-baseline --steps 120 --warmup 3 > gpurun_out/trace_l_bench.json 2> gpurun_out/trace_l.err || { echo TRACE_FAIL; exit 1; }
find gpurun_out/trace_l -name "*kernel_trace.csv" -exec cp {} gpurun_out/trace_l_kernels.csv \;
rm -rf gpurun_out/trace_l
python3 tools/trace_timeline.py gpurun_out/trace_l_kernels.csv > gpurun_out/timeline_s13.txt && head -80 gpurun_out/timeline_s13.txt
