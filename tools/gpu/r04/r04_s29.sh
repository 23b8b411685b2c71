# Round 4, session 29: split-bf16 GEMM with the A operand two k-tiles ahead (three register sets)
# vs two (TTAMM_GEMM_ADEEP=2): gemm_bench shapes, C2 bench, GEMM parity tests
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in 3 2; do
  if [ $v = 2 ]; then export TTAMM_GEMM_ADEEP=2; else unset TTAMM_GEMM_ADEEP; fi
  timeout -k 10 200 ./two-tower-augmented-with-adaptive-mimic-mechanism_amd/build/gemm_bench > gpurun_out/s29_gemm_ad$v.txt 2>&1 || { echo GB_FAIL; tail -5 gpurun_out/s29_gemm_ad$v.txt; exit 1; }
  echo "== ADEEP $v"; grep -E "fwd|dgrad" gpurun_out/s29_gemm_ad$v.txt | grep split
done
unset TTAMM_GEMM_ADEEP
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_step_parity_gpu.py tests/test_fullsize_parity_gpu.py -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/s29_tests.log 2>&1; rc=$?; grep -E "passed|failed|^FAILED|Error" gpurun_out/s29_tests.log | tail -5
if [ $rc -ne 0 ]; then echo "rc=$rc"; exit $rc; fi
for v in 3 2 3; do
  if [ $v = 2 ]; then export TTAMM_GEMM_ADEEP=2; else unset TTAMM_GEMM_ADEEP; fi
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/s29_c2.json 2> gpurun_out/s29_c2.err || { echo BENCH_FAIL; tail -5 gpurun_out/s29_c2.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/s29_c2.json')); print('C2 ADEEP=$v', d['value'], d['ms_per_step'], [(k['kernel'][:20], k.get('ms_per_step')) for k in d['kernels']])"
done
