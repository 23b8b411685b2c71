# Round 4, session 18: touched-row updates on the aux stream in the row-sharded TOWERS_BWD phase;
# aux events keyed by aux stream: sharded tests, emulated 8-rank C2 (look-ahead on / off) and C4
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_sharded_gpu.py tests/test_sharded_options_gpu.py -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/s18_sharded.log 2>&1; rc=$?; grep -E "passed|failed|^FAILED|Error" gpurun_out/s18_sharded.log | tail -8
if [ $rc -ne 0 ]; then echo "rc=$rc"; exit $rc; fi
for la in "" "--no-look-ahead"; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline --emulate-world 8 --steps 200 --warmup 5 $la > gpurun_out/s18_emu$la.json 2> gpurun_out/s18_emu$la.err || { echo EMU_FAIL; tail -20 gpurun_out/s18_emu$la.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/s18_emu$la.json')); print('emu8 $la', d['value'], d['ms_per_step'])"
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline --emulate-world 8 --config c4 --steps 30 --warmup 3 > gpurun_out/s18_c4emu.json 2> gpurun_out/s18_c4emu.err || { echo C4EMU_FAIL; tail -20 gpurun_out/s18_c4emu.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/s18_c4emu.json')); print('c4 emu8', d['value'], d['ms_per_step'])"
