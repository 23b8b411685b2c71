# final tree: full GPU suite, smoke, the driver's bench command, C5 and C4 lines, rocprofv3 stats of C2
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s36_gpu_tests.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s36_smoke.log 2>&1
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/s36_driver.json 2> gpurun_out/s36_driver.err
timeout -k 10 400 python bench.py --no-cpu-baseline --steps 20 --warmup 5 --config c5 > gpurun_out/s36_c5.json 2> gpurun_out/s36_c5.err
timeout -k 10 400 python bench.py --no-cpu-baseline --steps 20 --warmup 5 --config c4 --no-gather-bulk > gpurun_out/s36_c4.json 2> gpurun_out/s36_c4.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof36 -o run -- python3 bench.py --no-cpu-baseline --no-exact-line --steps 20 --warmup 5 > gpurun_out/s36_prof_bench.json 2> gpurun_out/s36_prof.err
find gpurun_out/prof36 -name "*kernel_stats.csv" -exec cp {} gpurun_out/s36_c2_kernel_stats.csv \;
rm -rf gpurun_out/prof36
