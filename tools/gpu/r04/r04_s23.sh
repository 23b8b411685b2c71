# Round 4, session 23: the round's measurement set on the current tree — smoke, the full GPU
# suite, the default C2 line (with the CPU baseline), its rocprofv3 kernel-trace --stats, and
# the C2 in-batch / C4 / C5 / C3 / emulated 8-rank C2 and C4 lines
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s23_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/s23_smoke.log; exit 1; }
tail -n 1 gpurun_out/s23_smoke.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/s23_tests.log 2>&1; rc=$?; grep -E "passed|failed|^FAILED|Error" gpurun_out/s23_tests.log | tail -8
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "suite rc=$rc"; exit $rc; fi
timeout -k 10 600 python -u bench.py > gpurun_out/s23_c2.json 2> gpurun_out/s23_c2.err || { echo BENCH_FAIL; tail -20 gpurun_out/s23_c2.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/s23_c2.json')); print('C2', d['value'], d['ms_per_step'], d['roofline'].get('frac'), d['cpu_baseline'])"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/s23_prof -o run -- python3 bench.py --no-cpu-baseline > gpurun_out/s23_c2_prof.json 2> gpurun_out/s23_c2_prof.err || { echo PROF_FAIL; tail -20 gpurun_out/s23_c2_prof.err; exit 1; }
find gpurun_out/s23_prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/s23_c2_kernel_stats.csv \;
rm -rf gpurun_out/s23_prof
head -n 6 gpurun_out/s23_c2_kernel_stats.csv | cut -c1-160
for cfg in "--negatives in-batch" "--config c4" "--config c5" "--emulate-world 8" "--emulate-world 8 --config c4 --steps 30 --warmup 3"; do
  tag=$(echo $cfg | tr -d ' -' | cut -c1-40)
  timeout -k 10 500 python -u bench.py --no-cpu-baseline $cfg > gpurun_out/s23_$tag.json 2> gpurun_out/s23_$tag.err || { echo BENCH_FAIL $cfg; tail -5 gpurun_out/s23_$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/s23_$tag.json')); print('$tag', d['value'], d['ms_per_step'], d['roofline'].get('frac'))"
done
timeout -k 10 300 python -u tools/bench_retrieval.py > gpurun_out/s23_c3.json 2> gpurun_out/s23_c3.err || { echo C3_FAIL; tail -5 gpurun_out/s23_c3.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/s23_c3.json')); print('C3', d['value'], d.get('roofline',{}).get('frac'))"
