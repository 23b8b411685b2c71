# Round 3 session 15: gate with LDS fragments read one k-tile ahead; both towers' ID-row gathers
# and weight pads in one launch each; vectorised candidate scoring (parity tests + bench + trace +
# the 50M x 128 gather bench)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_step_parity_gpu.py tests/test_kernels_gpu.py tests/test_golden_gpu.py tests/test_sharded_gpu.py tests/test_module_autograd_gpu.py tests/test_retrieval_gpu.py tests/test_c1_gpu.py -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_s15.log 2>&1
rc=$?
tail -15 gpurun_out/gpu_tests_s15.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc"; exit $rc; fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/b_s15.json 2> gpurun_out/b_s15.err || { echo B_FAIL; tail -5 gpurun_out/b_s15.err; exit 1; }
python3 -c "
import json
d=json.load(open('gpurun_out/b_s15.json')); print(d['value'], d['ms_per_step'], d['final_loss'])"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_l -o run -- python3 bench.py --no-cpu-baseline --steps 120 --warmup 3 > gpurun_out/trace_l_bench.json 2> gpurun_out/trace_l.err || { echo TRACE_FAIL; exit 1; }
find gpurun_out/trace_l -name "*kernel_trace.csv" -exec cp {} gpurun_out/trace_l_kernels.csv \;
rm -rf gpurun_out/trace_l
python3 tools/trace_timeline.py gpurun_out/trace_l_kernels.csv > gpurun_out/timeline_s15.txt && head -60 gpurun_out/timeline_s15.txt
timeout -k 10 400 python -u tools/bench_gather.py > gpurun_out/gather_s15.json 2> gpurun_out/gather_s15.err || { echo GATHER_FAIL; tail -5 gpurun_out/gather_s15.err; exit 1; }
python3 -c "
import json
d=json.load(open('gpurun_out/gather_s15.json')); print(json.dumps(d['results'], indent=1))"
