set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_x -o run -- python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 $BENCH_ARGS > gpurun_out/trace_x_bench.json 2> gpurun_out/trace_x.err
find gpurun_out/trace_x -name "*kernel_trace.csv" -exec cp {} gpurun_out/trace_x_kernels.csv \;
rm -rf gpurun_out/trace_x
