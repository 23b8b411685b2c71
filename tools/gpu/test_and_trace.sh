set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t3.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b3_c2.json 2> gpurun_out/b3_c2.err
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_c2 -o run -- python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 $BENCH_ARGS > gpurun_out/trace_c2_bench.json 2> gpurun_out/trace_c2.err
find gpurun_out/trace_c2 -name "*kernel_trace.csv" -exec cp {} gpurun_out/trace_c2_kernels.csv \;
rm -rf gpurun_out/trace_c2
