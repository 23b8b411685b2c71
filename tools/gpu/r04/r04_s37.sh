# Round 4, session 37: kernel-trace timelines after the chunked epilogues, narrow 32-k two-set tiles and the wider prologue grid
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in c2 c5; do
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_$c -o run -- python3 bench.py --config $c --no-cpu-baseline --steps 12 --warmup 3 > gpurun_out/s37_${c}_trace.json 2> gpurun_out/s37_${c}_trace.err || { echo TRACE_FAIL; tail -20 gpurun_out/s37_${c}_trace.err; exit 1; }
find gpurun_out/trace_$c -name "*kernel_trace.csv" -exec cp {} gpurun_out/s37_${c}_kernels.csv \;
rm -rf gpurun_out/trace_$c
python3 tools/trace_timeline.py gpurun_out/s37_${c}_kernels.csv > gpurun_out/s37_${c}_timeline.txt; head -3 gpurun_out/s37_${c}_timeline.txt
done
