# Round 4, session 9: the C2 deferred-vs-eager breakdown; retrieval with long blocked lists
# (lower-bound search past 64 items): tests, then C3 at 20 / 1000 / 5000 blocked
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/diag/deferred_c2.py > gpurun_out/s9_diag_c2.txt 2>&1; grep -v amdgpu.ids gpurun_out/s9_diag_c2.txt | tail -n 30
timeout -k 10 300 python -u -m pytest tests/test_retrieval_gpu.py -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/s9_retr.log 2>&1 || { tail -n 30 gpurun_out/s9_retr.log; exit 1; }
tail -n 2 gpurun_out/s9_retr.log
for nb in 20 1000 5000; do
  timeout -k 10 300 python -u tools/bench_retrieval.py --blocked $nb --cpu-queries 0 > gpurun_out/s9_c3_b$nb.json 2> gpurun_out/s9_c3_b$nb.err || { echo C3_FAIL $nb; tail -5 gpurun_out/s9_c3_b$nb.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/s9_c3_b$nb.json')); print('C3 blocked=$nb', d['value'])"
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_emu -o run -- python3 bench.py --no-cpu-baseline --steps 12 --warmup 3 --emulate-world 8 > gpurun_out/s9_emu_bench.json 2> gpurun_out/s9_emu.err || { echo TRACE_FAIL; tail -20 gpurun_out/s9_emu.err; exit 1; }
find gpurun_out/trace_emu -name "*kernel_trace.csv" -exec cp {} gpurun_out/s9_emu_kernels.csv \;
rm -rf gpurun_out/trace_emu
python3 tools/trace_timeline.py gpurun_out/s9_emu_kernels.csv > gpurun_out/s9_emu_timeline.txt; head -3 gpurun_out/s9_emu_timeline.txt
