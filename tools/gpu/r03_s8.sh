# Round 3 session 8: concat output_dim != embedding dim (step parity, module autograd, sharded),
# retrieval with 128-item tiles (tests + C3 bench)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_step_parity_gpu.py tests/test_module_autograd_gpu.py tests/test_sharded_options_gpu.py tests/test_retrieval_gpu.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_s8.log 2>&1
rc=$?
tail -25 gpurun_out/gpu_tests_s8.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc"; exit $rc; fi
timeout -k 10 300 python -u tools/bench_retrieval.py > gpurun_out/c3_split.json 2> gpurun_out/c3_split.err || { echo C3_FAIL; tail -5 gpurun_out/c3_split.err; exit 1; }
cat gpurun_out/c3_split.json

export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/b_fusedgate.json 2> gpurun_out/b_fusedgate.err || { echo B_FAIL; exit 1; }
TTAMM_GENERIC_GATE=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/b_genericgate.json 2> gpurun_out/b_genericgate.err || { echo BG_FAIL; tail -5 gpurun_out/b_genericgate.err; exit 1; }
python3 -c "
import json
for f in ('b_fusedgate','b_genericgate'):
    d=json.load(open('gpurun_out/'+f+'.json'))
    print(f, d['value'], d['ms_per_step'], d['final_loss'])
"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_l -o run -- python3 bench.py --no-cpu-baseline --steps 120 --warmup 3 > gpurun_out/trace_l_bench.json 2> gpurun_out/trace_l.err || { echo TRACE_FAIL; exit 1; }
find gpurun_out/trace_l -name "*kernel_trace.csv" -exec cp {} gpurun_out/trace_l_kernels.csv \;
rm -rf gpurun_out/trace_l
python3 tools/trace_timeline.py gpurun_out/trace_l_kernels.csv > gpurun_out/timeline_s9.txt && head -70 gpurun_out/timeline_s9.txt
echo "tests rc=$rc"
