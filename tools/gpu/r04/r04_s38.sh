# Round 4, session 38: split-K layer-1 forward for the in-batch steps (hidden_splitk_tail_kernel)
# and the wider step-prologue grid.  Parity first, then
# C2 / C2 in-batch / C4 / C5 (split-K on and off), then a C2 kernel trace against session 34's
mkdir -p gpurun_out
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_step_parity_gpu.py tests/test_inbatch_gpu.py tests/test_deferred_gpu.py tests/test_sharded_gpu.py tests/test_fullsize_parity_gpu.py > gpurun_out/s38_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/s38_tests.log; exit 1; }
tail -2 gpurun_out/s38_tests.log
b() {  # label, env, args
  local tag=$1 pre=$2; shift 2
  env $pre timeout -k 10 400 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/s38_x.json 2> gpurun_out/s38_x.err || { echo BENCH_FAIL $tag; tail -5 gpurun_out/s38_x.err; return 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/s38_x.json')); print('$tag', d['value'], d['ms_per_step'])"
}
b c2 "" && b c2_inbatch "" --negatives in-batch && b c2_inbatch_nosplit "TTAMM_GEMM_NO_SPLITK=1" --negatives in-batch \
  && b c4 "" --config c4 && b c4_nosplit "TTAMM_GEMM_NO_SPLITK=1" --config c4 && b c5 "" --config c5 && b c2 "" || exit 1
for c in c2; do
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_$c -o run -- python3 bench.py --config $c --no-cpu-baseline --steps 12 --warmup 3 > gpurun_out/s38_${c}_trace.json 2> gpurun_out/s38_${c}_trace.err || { echo TRACE_FAIL; exit 1; }
find gpurun_out/trace_$c -name "*kernel_trace.csv" -exec cp {} gpurun_out/s38_${c}_kernels.csv \;
rm -rf gpurun_out/trace_$c
done
python3 tools/kernel_means.py gpurun_out/s38_c2_kernels.csv gpurun_out/s34_c2_kernels.csv | head -24
