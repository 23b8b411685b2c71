# Round 3 session 11: replay with scalar-register constants vs the LDS ring (micro-benchmark),
# deferred/fullsize tests, default bench both ways
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
B=two-tower-augmented-with-adaptive-mimic-mechanism_amd/build
timeout -k 10 120 $B/replay_bench > gpurun_out/replay_bench_s.txt 2>&1 || { echo RB_FAIL; cat gpurun_out/replay_bench_s.txt; exit 1; }
TTAMM_REPLAY_LDS=1 timeout -k 10 120 $B/replay_bench > gpurun_out/replay_bench_lds.txt 2>&1 || { echo RB2_FAIL; exit 1; }
cat gpurun_out/replay_bench_s.txt gpurun_out/replay_bench_lds.txt
timeout -k 10 600 python -u -m pytest tests/test_deferred_gpu.py tests/test_fullsize_gpu.py tests/test_step_parity_gpu.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_s11.log 2>&1
rc=$?
tail -5 gpurun_out/gpu_tests_s11.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc"; exit $rc; fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/b_s11.json 2> gpurun_out/b_s11.err || { echo B_FAIL; tail -5 gpurun_out/b_s11.err; exit 1; }
TTAMM_REPLAY_LDS=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/b_s11_lds.json 2> gpurun_out/b_s11_lds.err || { echo B2_FAIL; exit 1; }
python3 -c "
import json
for f in ('b_s11','b_s11_lds'):
    d=json.load(open('gpurun_out/'+f+'.json')); r=d['roofline']
    print(f, d['value'], d['ms_per_step'], r['ms_per_step'], r.get('parts_ms_per_step'))
"
