# Round 3 session 26: retrieval with the hierarchical score filter and owner-wave compaction (one barrier per tile) (tests + C3 bench), then
# timing ablations of retrieval_x_kernel (TTAMM_RETRIEVAL_ABLATE: 1 no filter, 2 no MFMA,
# 4 no tile staging; results of ablated runs are wrong by construction, timing only)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_retrieval_gpu.py tests/test_c1_gpu.py -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_s26.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests_s26.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc"; exit $rc; fi
timeout -k 10 300 python -u tools/bench_retrieval.py > gpurun_out/c3_s26.json 2> gpurun_out/c3_s26.err || { echo C3_FAIL; tail -5 gpurun_out/c3_s26.err; exit 1; }
cat gpurun_out/c3_s26.json
for a in 1 2 4 3 6 7; do
  TTAMM_RETRIEVAL_ABLATE=$a timeout -k 10 200 python -u tools/bench_retrieval.py --cpu-queries 0 --reps 3 > gpurun_out/c3_s26_ab$a.json 2> gpurun_out/c3_s26_ab$a.err || { echo AB_FAIL $a; tail -5 gpurun_out/c3_s26_ab$a.err; exit 1; }
  echo "ablate $a: $(python3 -c "import json;d=json.load(open('gpurun_out/c3_s26_ab$a.json'));print(d['ms_per_batch'])")"
done
