# all GPU tests, the C2 / C5 bench lines, the bf16 GEMM micro-benchmark (developer script)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gt.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b_c2.json 2> gpurun_out/b_c2.err
timeout -k 10 300 python bench.py --no-cpu-baseline --config c5 > gpurun_out/b_c5.json 2> gpurun_out/b_c5.err
timeout -k 10 60 two-tower-augmented-with-adaptive-mimic-mechanism_amd/build/gemm_bench_bf16 > gpurun_out/gb16.txt 2>&1
