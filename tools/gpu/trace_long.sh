# kernel trace of a steady-state C2 run (120 timed steps; developer script)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_l -o run -- python3 bench.py --no-cpu-baseline --steps 120 --warmup 3 $BENCH_ARGS > gpurun_out/trace_l_bench.json 2> gpurun_out/trace_l.err
find gpurun_out/trace_l -name "*kernel_trace.csv" -exec cp {} gpurun_out/trace_l_kernels.csv \;
rm -rf gpurun_out/trace_l
