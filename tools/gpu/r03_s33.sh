# Round 3 session 33: short closing check: retrieval and C1 tests, the C3 bench line (roofline
# against the split-bf16 ceiling)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_retrieval_gpu.py tests/test_c1_gpu.py -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_s33.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests_s33.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc"; exit $rc; fi
timeout -k 10 300 python -u tools/bench_retrieval.py > gpurun_out/c3_s33.json 2> gpurun_out/c3_s33.err || { echo C3_FAIL; tail -5 gpurun_out/c3_s33.err; exit 1; }
cat gpurun_out/c3_s33.json
TTAMM_RETRIEVAL_ABLATE=1 timeout -k 10 200 python -u tools/bench_retrieval.py --cpu-queries 0 --reps 3 > gpurun_out/c3_s33_ab1.json 2> gpurun_out/c3_s33_ab1.err || { echo AB_FAIL; exit 1; }
timeout -k 10 200 python -u tools/bench_retrieval.py --cpu-queries 0 --reps 3 --blocked 0 > gpurun_out/c3_s33_nob.json 2> gpurun_out/c3_s33_nob.err || { echo NOB_FAIL; tail -5 gpurun_out/c3_s33_nob.err; exit 1; }
for f in ab1 nob; do echo "$f: $(python3 -c "import json;d=json.load(open('gpurun_out/c3_s33_$f.json'));print(d['ms_per_batch'])")"; done
