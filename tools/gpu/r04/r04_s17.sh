# Round 4, session 17: touched-row updates on the aux stream beside the MLP backward (one
# process): parity tests, C2 with / without (TTAMM_ROWS_MAIN=1), C2 in-batch, C4, C5
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_step_parity_gpu.py tests/test_deferred_gpu.py tests/test_optimizers_gpu.py tests/test_fullsize_parity_gpu.py tests/test_c1_gpu.py tests/test_data_gpu.py tests/test_inbatch_gpu.py -q -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/s17_tests.log 2>&1; rc=$?; grep -E "passed|failed|^FAILED|Error" gpurun_out/s17_tests.log | tail -8
if [ $rc -ne 0 ]; then echo "tests rc=$rc"; exit $rc; fi
for v in 0 1; do
  if [ $v = 1 ]; then export TTAMM_ROWS_MAIN=1; else unset TTAMM_ROWS_MAIN; fi
  timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/s17_c2_rm$v.json 2> gpurun_out/s17_c2_rm$v.err || { echo BENCH_FAIL; tail -5 gpurun_out/s17_c2_rm$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/s17_c2_rm$v.json')); print('C2 rows_main=$v', d['value'], d['ms_per_step'])"
done
unset TTAMM_ROWS_MAIN
for cfg in "--negatives in-batch" "--config c4" "--config c5"; do
  tag=$(echo $cfg | tr -d ' -')
  timeout -k 10 400 python -u bench.py --no-cpu-baseline $cfg > gpurun_out/s17_$tag.json 2> gpurun_out/s17_$tag.err || { echo BENCH_FAIL $cfg; tail -5 gpurun_out/s17_$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/s17_$tag.json')); print('$tag', d['value'], d['ms_per_step'])"
done
