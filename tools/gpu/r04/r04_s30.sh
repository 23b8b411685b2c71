# Round 4, session 30: forward GEMMs with A two k-tiles ahead (dgrad two sets): parity tests and
# the C2 / C2 in-batch / C4 / C5 / emulated 8-rank C2 lines
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_step_parity_gpu.py tests/test_fullsize_parity_gpu.py tests/test_golden_gpu.py tests/test_inbatch_gpu.py tests/test_sharded_gpu.py tests/test_module_autograd_gpu.py -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/s30_tests.log 2>&1; rc=$?; grep -E "passed|failed|^FAILED|Error" gpurun_out/s30_tests.log | tail -5
if [ $rc -ne 0 ]; then echo "rc=$rc"; exit $rc; fi
for pre in "" "TTAMM_WGRAD_ADEEP=3"; do for cfg in "" "--negatives in-batch" "--config c4" "--config c5" "--emulate-world 8 --steps 200 --warmup 5"; do
  tag=$(echo $cfg | tr -d ' -' | cut -c1-24)
  env $pre timeout -k 10 400 python -u bench.py --no-cpu-baseline $cfg > gpurun_out/s30_$tag.json 2> gpurun_out/s30_$tag.err || { echo BENCH_FAIL $cfg; tail -5 gpurun_out/s30_$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/s30_$tag.json')); print('[$pre] [$cfg]', d['value'], d['ms_per_step'])"
done; done
