# Round 3 session 16: the rolling slice started at the table updates (late) vs behind the grouping
# (TTAMM_SLICE_EARLY=1): deferred / full-size / step tests, bench A/B, steady-state trace
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_deferred_gpu.py tests/test_fullsize_gpu.py tests/test_step_parity_gpu.py tests/test_c1_gpu.py -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_s16.log 2>&1
rc=$?
tail -5 gpurun_out/gpu_tests_s16.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc"; exit $rc; fi
for v in late early late; do
  if [ $v = early ]; then export TTAMM_SLICE_EARLY=1; else unset TTAMM_SLICE_EARLY; fi
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/b_s16_$v.json 2> gpurun_out/b_s16_$v.err || { echo B_FAIL; tail -5 gpurun_out/b_s16_$v.err; exit 1; }
  python3 -c "
import json
d=json.load(open('gpurun_out/b_s16_$v.json')); r=d['roofline']; print('$v', d['value'], d['ms_per_step'], r['ms_per_step'], r.get('parts_ms_per_step'), d['final_loss'])"
done
unset TTAMM_SLICE_EARLY
for c in c4 c5; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --config $c > gpurun_out/b_s16_$c.json 2> gpurun_out/b_s16_$c.err || { echo B_FAIL; tail -5 gpurun_out/b_s16_$c.err; exit 1; }
  python3 -c "
import json
d=json.load(open('gpurun_out/b_s16_$c.json')); print('$c', d['value'], d['ms_per_step'], d['final_loss'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_l -o run -- python3 bench.py --no-cpu-baseline --steps 120 --warmup 3 > gpurun_out/trace_l_bench.json 2> gpurun_out/trace_l.err || { echo TRACE_FAIL; exit 1; }
find gpurun_out/trace_l -name "*kernel_trace.csv" -exec cp {} gpurun_out/trace_l_kernels.csv \;
rm -rf gpurun_out/trace_l
python3 tools/trace_timeline.py gpurun_out/trace_l_kernels.csv > gpurun_out/timeline_s16.txt && head -60 gpurun_out/timeline_s16.txt
