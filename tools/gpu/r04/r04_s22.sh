# Round 4, session 22: ordering experiments with the row updates on the aux stream — the narrow
# weight-gradient launch first (TTAMM_WGRAD_NARROW_FIRST), the slice behind the row updates
# (TTAMM_SLICE_AFTER_ROWS); deferred = eager with the latter
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TTAMM_SLICE_AFTER_ROWS=1 timeout -k 10 600 python -u -m pytest tests/test_deferred_gpu.py tests/test_step_parity_gpu.py -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/s22_tests.log 2>&1; rc=$?; grep -E "passed|failed|^FAILED|Error" gpurun_out/s22_tests.log | tail -5
if [ $rc -ne 0 ]; then echo "rc=$rc"; exit $rc; fi
for combo in "" "TTAMM_WGRAD_NARROW_FIRST=1" "TTAMM_SLICE_AFTER_ROWS=1" "TTAMM_WGRAD_NARROW_FIRST=1 TTAMM_SLICE_AFTER_ROWS=1"; do
  tag=$(echo "$combo" | tr -cd 'A-Z' | sed 's/TTAMM//g' | cut -c1-30)
  for cfg in "" "--config c4" "--emulate-world 8 --steps 200 --warmup 5"; do
    env $combo timeout -k 10 400 python -u bench.py --no-cpu-baseline $cfg > gpurun_out/s22_x.json 2> gpurun_out/s22_x.err || { echo BENCH_FAIL "$combo" "$cfg"; tail -5 gpurun_out/s22_x.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/s22_x.json')); print('[$combo] [$cfg]', d['value'], d['ms_per_step'])"
  done
done
