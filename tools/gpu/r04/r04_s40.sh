# Round 4, session 40: the rebuilt round-end library (split-K reverted) — smoke, the C1 tests,
# the default C2 line
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s40_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/s40_smoke.log; exit 1; }
tail -n 1 gpurun_out/s40_smoke.log
timeout -k 10 600 python -u -m pytest tests/test_c1_gpu.py -q -p no:cacheprovider --timeout 500 --timeout-method thread > gpurun_out/s40_c1.log 2>&1 || { echo C1_FAIL; tail -30 gpurun_out/s40_c1.log; exit 1; }
tail -n 1 gpurun_out/s40_c1.log
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/s40_c2.json 2> gpurun_out/s40_c2.err || { echo BENCH_FAIL; tail -20 gpurun_out/s40_c2.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/s40_c2.json')); print('C2', d['value'], d['ms_per_step'])"
