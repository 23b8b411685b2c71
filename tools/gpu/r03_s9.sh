# Round 3 session 9: fused vs generic (split-bf16 GEMM) gate on the default bench; a steady-state
# kernel trace (120 timed steps) for the step timeline
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
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
