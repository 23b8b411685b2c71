# Round 4, session 7 (combined): pipelined in-batch kernel vs split kernel + its tests; the fast
# g = 0 replay (deferred tests, isolated replay, C2 bench); autograd / retrieval fixes; C3 with long
# blocked lists; the emulated 8-rank C2 step and its host profile
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in x p; do
  for pos in 65536 8192; do
    TTAMM_IB_KERNEL=$v timeout -k 10 120 python -u tools/bench_inbatch.py --positives $pos > gpurun_out/s7_ib_${v}_$pos.json 2> gpurun_out/s7_ib_${v}_$pos.err || { echo IB_FAIL $v $pos; tail -20 gpurun_out/s7_ib_${v}_$pos.err; exit 1; }
    echo "$v $pos $(cat gpurun_out/s7_ib_${v}_$pos.json)"
  done
done
TTAMM_IB_KERNEL=p timeout -k 10 600 python -u -m pytest tests/test_inbatch_op_gpu.py tests/test_inbatch_gpu.py -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/s7_ib_tests.log 2>&1; tail -3 gpurun_out/s7_ib_tests.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -s -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/s7_tests.log 2>&1; rc=$?; grep -E "passed|failed|near ties|fast vs exact|^FAILED|Error" gpurun_out/s7_tests.log | tail -25
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "suite rc=$rc"; exit $rc; fi
timeout -k 10 120 ./two-tower-augmented-with-adaptive-mimic-mechanism_amd/build/replay_bench > gpurun_out/s7_replay_bench.txt 2>&1; cat gpurun_out/s7_replay_bench.txt | tail -8
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/s7_bench.json 2> gpurun_out/s7_bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/s7_bench.err; exit 1; }
python3 -c "
import json
d=json.load(open('gpurun_out/s7_bench.json')); print('C2', d['value'], d['ms_per_step']); r=d['roofline']; print(r['kernel'][:40], r['ms_per_step'], r.get('parts_ms_per_step'), r.get('frac'))"
for nb in 20 1000 5000; do
  timeout -k 10 300 python -u tools/bench_retrieval.py --blocked $nb --cpu-queries 0 > gpurun_out/s7_c3_b$nb.json 2> gpurun_out/s7_c3_b$nb.err || { echo C3_FAIL $nb; tail -5 gpurun_out/s7_c3_b$nb.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/s7_c3_b$nb.json')); print('C3 blocked=$nb', d['value'])"
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline --emulate-world 8 --steps 100 --warmup 3 > gpurun_out/s7_emu.json 2> gpurun_out/s7_emu.err || { echo EMU_FAIL; tail -20 gpurun_out/s7_emu.err; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline --emulate-world 8 --steps 100 --warmup 3 --no-look-ahead > gpurun_out/s7_emu_nola.json 2> gpurun_out/s7_emu_nola.err || { echo EMU2_FAIL; tail -20 gpurun_out/s7_emu_nola.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/s7_emu_nola.json')); print('emu8 no look-ahead', d['value'], d['ms_per_step'])"
python3 -c "import json; d=json.load(open('gpurun_out/s7_emu.json')); print('emu8', d['value'], d['ms_per_step'])"
timeout -k 10 300 python -u -m cProfile -o gpurun_out/s7_emu.prof bench.py --no-cpu-baseline --emulate-world 8 --steps 100 --warmup 3 > gpurun_out/s7_emu_prof.json 2> gpurun_out/s7_emu_prof.err || { echo PROF_FAIL; tail -20 gpurun_out/s7_emu_prof.err; exit 1; }
python3 -c "
import pstats
p = pstats.Stats('gpurun_out/s7_emu.prof'); p.sort_stats('tottime').print_stats(40)" > gpurun_out/s7_prof_tottime.txt
python3 -c "
import pstats
p = pstats.Stats('gpurun_out/s7_emu.prof'); p.sort_stats('cumulative').print_stats(50)" > gpurun_out/s7_prof_cum.txt
echo done
for wt in 0 1; do
  if [ $wt = 1 ]; then export TTAMM_GEMM_WIDE_TILES=1; else unset TTAMM_GEMM_WIDE_TILES; fi
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --negatives in-batch > gpurun_out/s7_c2ib_wt$wt.json 2> gpurun_out/s7_c2ib_wt$wt.err || { echo IB_BENCH_FAIL; tail -5 gpurun_out/s7_c2ib_wt$wt.err; exit 1; }
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --config c4 > gpurun_out/s7_c4_wt$wt.json 2> gpurun_out/s7_c4_wt$wt.err || { echo C4_FAIL; tail -5 gpurun_out/s7_c4_wt$wt.err; exit 1; }
  python3 -c "
import json
for f in ('s7_c2ib_wt$wt','s7_c4_wt$wt'):
    d=json.load(open('gpurun_out/'+f+'.json')); print(f, d['value'], d['ms_per_step'], [(k['kernel'][:30], k.get('ms_per_step')) for k in d['kernels']])"
done
unset TTAMM_GEMM_WIDE_TILES
