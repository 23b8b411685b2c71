# Round 3 session 22: grid-stride fused prologue (64 blocks per part); the gate with its output
# stores ablated (TTAMM_GATE_ABLATE=1, timing only); tests of the prologue paths; bench; trace
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_fullsize_gpu.py tests/test_deferred_gpu.py tests/test_index_errors_gpu.py tests/test_step_parity_gpu.py tests/test_sharded_gpu.py tests/test_c1_gpu.py -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_s22.log 2>&1
rc=$?
tail -4 gpurun_out/gpu_tests_s22.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc"; exit $rc; fi
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/b_s22_$i.json 2> gpurun_out/b_s22_$i.err || { echo B_FAIL; tail -5 gpurun_out/b_s22_$i.err; exit 1; }
  python3 -c "
import json
d=json.load(open('gpurun_out/b_s22_$i.json')); r=d['roofline']; print('$i', d['value'], d['ms_per_step'], r['ms_per_step'], d['final_loss'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_l -o run -- python3 bench.py --no-cpu-baseline --steps 120 --warmup 3 > gpurun_out/trace_l_bench.json 2> gpurun_out/trace_l.err || { echo TRACE_FAIL; exit 1; }
find gpurun_out/trace_l -name "*kernel_trace.csv" -exec cp {} gpurun_out/trace_l_kernels.csv \;
rm -rf gpurun_out/trace_l
python3 tools/trace_timeline.py gpurun_out/trace_l_kernels.csv > gpurun_out/timeline_s22.txt && head -12 gpurun_out/timeline_s22.txt
export TTAMM_GATE_ABLATE=1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_a -o run -- python3 bench.py --no-cpu-baseline --steps 60 --warmup 3 > gpurun_out/trace_a_bench.json 2> gpurun_out/trace_a.err || { echo TRACEA_FAIL; exit 1; }
find gpurun_out/trace_a -name "*kernel_trace.csv" -exec cp {} gpurun_out/trace_a_kernels.csv \;
rm -rf gpurun_out/trace_a
python3 tools/trace_timeline.py gpurun_out/trace_a_kernels.csv > gpurun_out/timeline_s22_ablate.txt && grep -E "gate_(fwd|bwd)" gpurun_out/timeline_s22_ablate.txt
