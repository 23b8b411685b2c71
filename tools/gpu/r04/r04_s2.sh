# Round 4, session 2: VALU issue rates incl. VOP2 forms, the in-batch op at the C2 / C4-rank shapes
# vs fp64, the optimizer tests, then the whole GPU suite, the C2 bench and the C4 emulated 8-rank line
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 ./two-tower-augmented-with-adaptive-mimic-mechanism_amd/build/valu_bench > gpurun_out/s2_valu.txt 2>&1 || { echo VALU_FAIL; cat gpurun_out/s2_valu.txt; exit 1; }
cat gpurun_out/s2_valu.txt
timeout -k 10 600 python -u -m pytest tests/test_inbatch_op_gpu.py tests/test_optimizers_gpu.py -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/s2_new.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/s2_new.log | tail -40
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "new tests rc=$rc"; exit $rc; fi
timeout -k 10 1500 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 800 --timeout-method thread > gpurun_out/s2_gpu_tests.log 2>&1
rc2=$?
tail -15 gpurun_out/s2_gpu_tests.log
if [ $rc2 -ne 0 ] && [ $rc2 -ne 1 ]; then echo "suite rc=$rc2"; exit $rc2; fi
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/s2_bench.json 2> gpurun_out/s2_bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/s2_bench.err; exit 1; }
python3 -c "
import json
d=json.load(open('gpurun_out/s2_bench.json')); print('C2', d['value'], d['ms_per_step'])"
timeout -k 10 400 python -u bench.py --config c4 --emulate-world 8 --steps 40 --warmup 3 > gpurun_out/s2_c4_emu8.json 2> gpurun_out/s2_c4_emu8.err || { echo EMU_FAIL; tail -20 gpurun_out/s2_c4_emu8.err; exit 1; }
python3 -c "
import json
d=json.load(open('gpurun_out/s2_c4_emu8.json'))
print('C4emu8', d['value'], d['ms_per_step'])
for k in d['kernels']: print(k['kernel'][:60], k.get('ms_per_step'), k.get('frac'))"
echo "rc new=$rc suite=$rc2"
