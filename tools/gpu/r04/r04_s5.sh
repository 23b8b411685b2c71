# Round 4, session 5: host-side profile of the emulated 8-rank C2 step (cProfile), and the same
# bench without the profiler
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --no-cpu-baseline --emulate-world 8 --steps 100 --warmup 3 > gpurun_out/s5_emu.json 2> gpurun_out/s5_emu.err || { echo EMU_FAIL; tail -20 gpurun_out/s5_emu.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/s5_emu.json')); print('emu8', d['value'], d['ms_per_step'])"
timeout -k 10 300 python -u -m cProfile -o gpurun_out/s5_emu.prof bench.py --no-cpu-baseline --emulate-world 8 --steps 100 --warmup 3 > gpurun_out/s5_emu_prof.json 2> gpurun_out/s5_emu_prof.err || { echo PROF_FAIL; tail -20 gpurun_out/s5_emu_prof.err; exit 1; }
python3 -c "
import pstats
p = pstats.Stats('gpurun_out/s5_emu.prof'); p.sort_stats('tottime').print_stats(35)" > gpurun_out/s5_prof_tottime.txt
python3 -c "
import pstats
p = pstats.Stats('gpurun_out/s5_emu.prof'); p.sort_stats('cumulative').print_stats(45)" > gpurun_out/s5_prof_cum.txt
head -60 gpurun_out/s5_prof_tottime.txt
timeout -k 10 600 python -u -m pytest tests/test_deferred_gpu.py -v -s -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/s5_deferred.log 2>&1; grep -E "PASSED|FAILED|fast vs exact" gpurun_out/s5_deferred.log | tail -20
timeout -k 10 120 ./two-tower-augmented-with-adaptive-mimic-mechanism_amd/build/replay_bench > gpurun_out/s5_replay_bench.txt 2>&1; cat gpurun_out/s5_replay_bench.txt
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/s5_bench.json 2> gpurun_out/s5_bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/s5_bench.err; exit 1; }
python3 -c "
import json
d=json.load(open('gpurun_out/s5_bench.json')); print('C2', d['value'], d['ms_per_step']); r=d['roofline']; print(r['kernel'][:40], r['ms_per_step'], r.get('parts_ms_per_step'), r.get('frac'))"
timeout -k 10 600 python -u -m pytest tests/test_module_autograd_gpu.py tests/test_retrieval_gpu.py -q -s -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/s5_tests.log 2>&1; grep -E "passed|failed|near ties|Error" gpurun_out/s5_tests.log | tail -8
for nb in 20 1000 5000; do
  timeout -k 10 300 python -u tools/bench_retrieval.py --blocked $nb --cpu-queries 0 > gpurun_out/s5_c3_b$nb.json 2> gpurun_out/s5_c3_b$nb.err || { echo C3_FAIL $nb; tail -5 gpurun_out/s5_c3_b$nb.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/s5_c3_b$nb.json')); print('C3 blocked=$nb', d['value'])"
done
