# Round 3 session 21: staging + sampler + step count / AdamW constants in one launch (the
# step's prologue), row updates with three float4 per lane at D = 96: the whole GPU suite, then
# the default bench A/B (TTAMM_ROW_UPDATE_POW2=1: the previous row-update kernel) and a trace
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1500 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/gpu_tests_s21.log 2>&1
rc=$?
tail -8 gpurun_out/gpu_tests_s21.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc"; exit $rc; fi
for i in 1 2 3 4; do
  if [ $i = 2 ] || [ $i = 4 ]; then export TTAMM_ROW_UPDATE_POW2=1; else unset TTAMM_ROW_UPDATE_POW2; fi
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/b_s21_$i.json 2> gpurun_out/b_s21_$i.err || { echo B_FAIL; tail -5 gpurun_out/b_s21_$i.err; exit 1; }
  python3 -c "
import json
d=json.load(open('gpurun_out/b_s21_$i.json')); r=d['roofline']; print('$i', d['value'], d['ms_per_step'], r['ms_per_step'], r.get('parts_ms_per_step'), d['final_loss'])"
done
unset TTAMM_ROW_UPDATE_POW2
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_l -o run -- python3 bench.py --no-cpu-baseline --steps 120 --warmup 3 > gpurun_out/trace_l_bench.json 2> gpurun_out/trace_l.err || { echo TRACE_FAIL; exit 1; }
find gpurun_out/trace_l -name "*kernel_trace.csv" -exec cp {} gpurun_out/trace_l_kernels.csv \;
rm -rf gpurun_out/trace_l
python3 tools/trace_timeline.py gpurun_out/trace_l_kernels.csv > gpurun_out/timeline_s21.txt && head -52 gpurun_out/timeline_s21.txt
