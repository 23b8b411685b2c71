# Round 4, session 44: in-batch planning at 256 blocks per role by default — smoke, the full GPU
# suite, C4 / C2 in-batch / C2 lines
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s44_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/s44_smoke.log; exit 1; }
tail -n 1 gpurun_out/s44_smoke.log
timeout -k 10 800 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/s44_tests.log 2>&1; rc=$?; grep -E "passed|failed|^FAILED|Error" gpurun_out/s44_tests.log | tail -8
if [ $rc -ne 0 ]; then echo "suite rc=$rc"; exit $rc; fi
for cfg in "--config c4" "--negatives in-batch" ""; do
  timeout -k 10 400 python -u bench.py --no-cpu-baseline $cfg > gpurun_out/s44_x.json 2> gpurun_out/s44_x.err || { echo BENCH_FAIL; tail -5 gpurun_out/s44_x.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/s44_x.json')); print('[$cfg]', d['value'], d['ms_per_step'], [round(k.get('frac') or 0, 3) for k in d.get('kernels', [])])"
done
