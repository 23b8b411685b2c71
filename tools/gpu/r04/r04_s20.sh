# Round 4, session 20: the ID-row gather on the aux stream beside the first-layer GEMM: parity
# (one process, sharded, options), C2 with / without (TTAMM_GATHER_MAIN=1), C4, emulated 8-rank C2
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_step_parity_gpu.py tests/test_deferred_gpu.py tests/test_sharded_gpu.py tests/test_sharded_options_gpu.py tests/test_fullsize_parity_gpu.py tests/test_c1_gpu.py -q -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/s20_tests.log 2>&1; rc=$?; grep -E "passed|failed|^FAILED|Error|no tests ran" gpurun_out/s20_tests.log | tail -8
if [ $rc -ne 0 ]; then echo "tests rc=$rc"; exit $rc; fi
for v in 0 1; do
  if [ $v = 1 ]; then export TTAMM_GATHER_MAIN=1; else unset TTAMM_GATHER_MAIN; fi
  timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/s20_c2_gm$v.json 2> gpurun_out/s20_c2_gm$v.err || { echo BENCH_FAIL; tail -5 gpurun_out/s20_c2_gm$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/s20_c2_gm$v.json')); print('C2 gather_main=$v', d['value'], d['ms_per_step'])"
done
unset TTAMM_GATHER_MAIN
timeout -k 10 400 python -u bench.py --no-cpu-baseline --config c4 > gpurun_out/s20_c4.json 2> gpurun_out/s20_c4.err || { echo C4_FAIL; tail -5 gpurun_out/s20_c4.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/s20_c4.json')); print('C4', d['value'], d['ms_per_step'])"
timeout -k 10 300 python -u bench.py --no-cpu-baseline --emulate-world 8 --steps 200 --warmup 5 > gpurun_out/s20_emu.json 2> gpurun_out/s20_emu.err || { echo EMU_FAIL; tail -20 gpurun_out/s20_emu.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/s20_emu.json')); print('emu8', d['value'], d['ms_per_step'])"
