# Round 4, session 16: look-ahead device work on its own stream (count exchange after the
# backward exchange): sharded tests, emulated 8-rank C2 with / without look-ahead, host profile
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_sharded_gpu.py tests/test_sharded_options_gpu.py -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/s16_sharded.log 2>&1; rc=$?; grep -E "passed|failed|^FAILED|Error" gpurun_out/s16_sharded.log | tail -8
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "rc=$rc"; exit $rc; fi
for la in "" "--no-look-ahead"; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline --emulate-world 8 --steps 200 --warmup 5 $la > gpurun_out/s16_emu$la.json 2> gpurun_out/s16_emu$la.err || { echo EMU_FAIL; tail -20 gpurun_out/s16_emu$la.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/s16_emu$la.json')); print('emu8 $la', d['value'], d['ms_per_step'])"
done
timeout -k 10 300 python -u tools/prof_host.py --steps 200 > gpurun_out/s16_prof_host.txt 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/s16_prof_host.txt; exit 1; }
head -n 12 gpurun_out/s16_prof_host.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_emu -o run -- python3 bench.py --no-cpu-baseline --steps 12 --warmup 3 --emulate-world 8 > gpurun_out/s16_emu_trace.json 2> gpurun_out/s16_emu_trace.err || { echo TRACE_FAIL; tail -20 gpurun_out/s16_emu_trace.err; exit 1; }
find gpurun_out/trace_emu -name "*kernel_trace.csv" -exec cp {} gpurun_out/s16_emu_kernels.csv \;
rm -rf gpurun_out/trace_emu
python3 tools/trace_timeline.py gpurun_out/s16_emu_kernels.csv > gpurun_out/s16_emu_timeline.txt; head -3 gpurun_out/s16_emu_timeline.txt
