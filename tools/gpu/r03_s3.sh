# Round 3 session 3: smoke, full GPU suite, default bench, emulated W=8 benches
# emulated W=8 per-rank benches (C4 in-batch Bg=65,536; C2).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/smoke.log; exit 1; }
timeout -k 10 1700 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 900 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -40 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
timeout -k 10 600 python -u bench.py > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || { echo BENCH_FAIL; tail -20 gpurun_out/bench_c2.err; exit 1; }
cat gpurun_out/bench_c2.json
timeout -k 10 400 python -u bench.py --config c4 --emulate-world 8 --steps 40 --warmup 3 > gpurun_out/bench_c4_emu8.json 2> gpurun_out/bench_c4_emu8.err || { echo EMU_FAIL; tail -20 gpurun_out/bench_c4_emu8.err; exit 1; }
cat gpurun_out/bench_c4_emu8.json
timeout -k 10 400 python -u bench.py --config c2 --emulate-world 8 --steps 100 --warmup 3 > gpurun_out/bench_c2_emu8.json 2> gpurun_out/bench_c2_emu8.err || { echo EMU2_FAIL; tail -20 gpurun_out/bench_c2_emu8.err; exit 1; }
cat gpurun_out/bench_c2_emu8.json
echo "pytest rc=$rc"
