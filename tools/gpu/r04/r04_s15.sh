# Round 4, session 15: full GPU suite after the packed-operand fix (no SLP in rows/optim/cal,
# pair constants in the fast replay, lower-bound blocked test); C2 bench; host cost of the
# emulated 8-rank step
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -s -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/s15_tests.log 2>&1; rc=$?; grep -E "passed|failed|^FAILED|Error" gpurun_out/s15_tests.log | tail -12
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "suite rc=$rc"; exit $rc; fi
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/s15_bench.json 2> gpurun_out/s15_bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/s15_bench.err; exit 1; }
python3 -c "
import json
d=json.load(open('gpurun_out/s15_bench.json')); print('C2', d['value'], d['ms_per_step']); print([(k['kernel'][:30], k.get('ms_per_step')) for k in d['kernels']])"
timeout -k 10 300 python -u bench.py --no-cpu-baseline --emulate-world 8 --steps 100 --warmup 3 > gpurun_out/s15_emu.json 2> gpurun_out/s15_emu.err || { echo EMU_FAIL; tail -20 gpurun_out/s15_emu.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/s15_emu.json')); print('emu8', d['value'], d['ms_per_step'])"
timeout -k 10 300 python -u tools/prof_host.py --steps 200 > gpurun_out/s15_prof_host.txt 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/s15_prof_host.txt; exit 1; }
head -n 30 gpurun_out/s15_prof_host.txt
