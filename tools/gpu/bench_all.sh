# C2 sampled / C5 / C2 exact-MFMA bench lines + a C2 kernel trace (developer script)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b_c2.json 2> gpurun_out/b_c2.err
timeout -k 10 300 python bench.py --no-cpu-baseline --config c5 > gpurun_out/b_c5.json 2> gpurun_out/b_c5.err
TTAMM_FP32_MFMA=exact timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b_c2_exact.json 2> gpurun_out/b_c2_exact.err
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_c2 -o run -- python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/trace_c2_bench.json 2> gpurun_out/trace_c2.err
find gpurun_out/trace_c2 -name "*kernel_trace.csv" -exec cp {} gpurun_out/trace_c2_kernels.csv \;
rm -rf gpurun_out/trace_c2
