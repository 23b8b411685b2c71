# Round 3 session 6: split-bf16 retrieval (tests + C3 bench, fp32 kernel beside it), the
# rewritten score kernel (step parity + sharded tests), aux-stream priority A/B on the bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_retrieval_gpu.py tests/test_step_parity_gpu.py tests/test_sharded_gpu.py tests/test_inbatch_gpu.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_s6.log 2>&1
rc=$?
tail -15 gpurun_out/gpu_tests_s6.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc"; exit $rc; fi
timeout -k 10 300 python -u tools/bench_retrieval.py > gpurun_out/c3_split.json 2> gpurun_out/c3_split.err || { echo C3_FAIL; tail -5 gpurun_out/c3_split.err; exit 1; }
cat gpurun_out/c3_split.json
TTAMM_RETRIEVAL_FP32=1 timeout -k 10 300 python -u tools/bench_retrieval.py > gpurun_out/c3_fp32.json 2> gpurun_out/c3_fp32.err || { echo C3F_FAIL; exit 1; }
cat gpurun_out/c3_fp32.json
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/b_prio0.json 2> gpurun_out/b_prio0.err || { echo B0_FAIL; exit 1; }
TTAMM_AUX_PRIORITY=-1 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/b_prio1.json 2> gpurun_out/b_prio1.err || { echo B1_FAIL; tail -5 gpurun_out/b_prio1.err; exit 1; }
python3 -c "
import json
for f in ('b_prio0','b_prio1'):
    d=json.load(open('gpurun_out/'+f+'.json')); r=d['roofline']
    print(f, d['value'], d['ms_per_step'], r['ms_per_step'], r.get('parts_ms_per_step'), [ (k['kernel'][:30], k.get('avg_launch_ms')) for k in d['kernels'][1:]])
"
