# Round 4, session 35: the per-kernel timing events' own cost (bench --kernel-events none) at C2,
# C4 and C5, and a kernel-trace timeline of C2 without them
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # tag, args
  local tag=$1; shift
  timeout -k 10 240 python3 bench.py --no-cpu-baseline "$@" > gpurun_out/s35_$tag.json 2> gpurun_out/s35_$tag.err || { echo "FAIL $tag"; tail -5 gpurun_out/s35_$tag.err; return 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/s35_$tag.json')); print('$tag', d['value'], d['ms_per_step'])"
}
for rep in 1 2; do
  run c2_ev$rep && run c2_none$rep --kernel-events none || exit 1
done
run c4_ev --config c4 && run c4_none --config c4 --kernel-events none || exit 1
run c5_ev --config c5 && run c5_none --config c5 --kernel-events none || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_c2n -o run -- python3 bench.py --no-cpu-baseline --kernel-events none --steps 12 --warmup 3 > gpurun_out/s35_c2n_trace.json 2> gpurun_out/s35_c2n_trace.err || { echo TRACE_FAIL; exit 1; }
find gpurun_out/trace_c2n -name "*kernel_trace.csv" -exec cp {} gpurun_out/s35_c2n_kernels.csv \;
rm -rf gpurun_out/trace_c2n
python3 tools/trace_timeline.py gpurun_out/s35_c2n_kernels.csv > gpurun_out/s35_c2n_timeline.txt; head -3 gpurun_out/s35_c2n_timeline.txt
