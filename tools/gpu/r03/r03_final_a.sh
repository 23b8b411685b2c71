# Round 3 final, part A: smoke, the whole GPU suite, the default bench with the CPU baseline, its
# rocprofv3 kernel stats, the C3 retrieval bench, c4 / c5 and emulated 8-rank benches
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fa_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/fa_smoke.log; exit 1; }
cat gpurun_out/fa_smoke.log | tail -1
timeout -k 10 1500 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/fa_gpu_tests.log 2>&1
rc=$?
tail -6 gpurun_out/fa_gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
timeout -k 10 600 python -u bench.py > gpurun_out/fa_bench.json 2> gpurun_out/fa_bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/fa_bench.err; exit 1; }
cat gpurun_out/fa_bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/stats -o run -- python3 bench.py --no-cpu-baseline > gpurun_out/stats_bench.json 2> gpurun_out/stats.err || { echo STATS_FAIL; exit 1; }
find gpurun_out/stats -name "*kernel_stats.csv" -exec cp {} gpurun_out/stats_kernel_stats.csv \;
rm -rf gpurun_out/stats
timeout -k 10 300 python -u tools/bench_retrieval.py > gpurun_out/fa_c3.json 2> gpurun_out/fa_c3.err || { echo C3_FAIL; tail -5 gpurun_out/fa_c3.err; exit 1; }
cat gpurun_out/fa_c3.json
timeout -k 10 400 python -u bench.py --no-cpu-baseline --negatives in-batch > gpurun_out/fa_c2_inbatch.json 2> gpurun_out/fa_c2_inbatch.err || { echo IB_FAIL; tail -5 gpurun_out/fa_c2_inbatch.err; exit 1; }
timeout -k 10 400 python -u bench.py --no-cpu-baseline --exact-table-math > gpurun_out/fa_c2_exact.json 2> gpurun_out/fa_c2_exact.err || { echo EX_FAIL; tail -5 gpurun_out/fa_c2_exact.err; exit 1; }
for c in c4 c5; do
  timeout -k 10 400 python -u bench.py --config $c --no-cpu-baseline > gpurun_out/fa_$c.json 2> gpurun_out/fa_$c.err || { echo ${c}_FAIL; tail -5 gpurun_out/fa_$c.err; exit 1; }
done
timeout -k 10 400 python -u bench.py --config c4 --emulate-world 8 --steps 40 --warmup 3 > gpurun_out/fa_c4_emu8.json 2> gpurun_out/fa_c4_emu8.err || { echo EMU_FAIL; tail -20 gpurun_out/fa_c4_emu8.err; exit 1; }
timeout -k 10 400 python -u bench.py --config c2 --emulate-world 8 --steps 100 --warmup 3 > gpurun_out/fa_c2_emu8.json 2> gpurun_out/fa_c2_emu8.err || { echo EMU2_FAIL; tail -20 gpurun_out/fa_c2_emu8.err; exit 1; }
python3 -c "
import json
for f in ('fa_c2_inbatch','fa_c2_exact','fa_c4','fa_c5','fa_c4_emu8','fa_c2_emu8'):
    d=json.load(open('gpurun_out/'+f+'.json')); print(f, d['value'], d['ms_per_step'], d['roofline']['kernel'][:40], d['roofline'].get('frac'))"
echo "pytest rc=$rc"
