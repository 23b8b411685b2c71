# Round 3 session 20: the rolling slice enqueued once the gate backward is (default) vs behind the
# grouping (TTAMM_SLICE_POINT=prologue): deferred / step tests, bench A/B, steady-state trace
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_deferred_gpu.py tests/test_step_parity_gpu.py tests/test_fullsize_gpu.py tests/test_c1_gpu.py -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_s20.log 2>&1
rc=$?
tail -5 gpurun_out/gpu_tests_s20.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc"; exit $rc; fi
for v in gate prologue gate prologue; do
  timeout -k 10 300 env TTAMM_SLICE_POINT=$v python -u bench.py --no-cpu-baseline > gpurun_out/b_s20_$v.json 2> gpurun_out/b_s20_$v.err || { echo B_FAIL; tail -5 gpurun_out/b_s20_$v.err; exit 1; }
  python3 -c "
import json
d=json.load(open('gpurun_out/b_s20_$v.json')); r=d['roofline']; print('$v', d['value'], d['ms_per_step'], r['ms_per_step'], r.get('parts_ms_per_step'))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_l -o run -- python3 bench.py --no-cpu-baseline --steps 120 --warmup 3 > gpurun_out/trace_l_bench.json 2> gpurun_out/trace_l.err || { echo TRACE_FAIL; exit 1; }
find gpurun_out/trace_l -name "*kernel_trace.csv" -exec cp {} gpurun_out/trace_l_kernels.csv \;
rm -rf gpurun_out/trace_l
python3 tools/trace_timeline.py gpurun_out/trace_l_kernels.csv > gpurun_out/timeline_s20.txt && head -50 gpurun_out/timeline_s20.txt
