# Round 4, session 19: kernel-trace timeline of the one-process C2 step with the row updates on
# the aux stream
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_c2 -o run -- python3 bench.py --no-cpu-baseline --steps 12 --warmup 3 > gpurun_out/s19_c2_trace.json 2> gpurun_out/s19_c2_trace.err || { echo TRACE_FAIL; tail -20 gpurun_out/s19_c2_trace.err; exit 1; }
find gpurun_out/trace_c2 -name "*kernel_trace.csv" -exec cp {} gpurun_out/s19_c2_kernels.csv \;
rm -rf gpurun_out/trace_c2
python3 tools/trace_timeline.py gpurun_out/s19_c2_kernels.csv > gpurun_out/s19_c2_timeline.txt; head -3 gpurun_out/s19_c2_timeline.txt
