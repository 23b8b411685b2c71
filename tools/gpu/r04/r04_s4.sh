# Round 4, session 4: in-batch kernel with the label-free fast path, kernel-trace timeline of the
# emulated 8-rank C2 step
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/bench_inbatch.py > gpurun_out/s4_ib.json 2> gpurun_out/s4_ib.err || { echo IB_FAIL; tail -20 gpurun_out/s4_ib.err; exit 1; }
cat gpurun_out/s4_ib.json
timeout -k 10 120 python -u tools/bench_inbatch.py --positives 8192 > gpurun_out/s4_ib_c2.json 2>&1 && cat gpurun_out/s4_ib_c2.json
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_emu -o run -- python3 bench.py --no-cpu-baseline --steps 12 --warmup 3 --emulate-world 8 > gpurun_out/s4_emu_bench.json 2> gpurun_out/s4_emu.err || { echo TRACE_FAIL; tail -20 gpurun_out/s4_emu.err; exit 1; }
find gpurun_out/trace_emu -name "*kernel_trace.csv" -exec cp {} gpurun_out/s4_emu_kernels.csv \;
rm -rf gpurun_out/trace_emu
python3 tools/trace_timeline.py gpurun_out/s4_emu_kernels.csv > gpurun_out/s4_emu_timeline.txt; head -5 gpurun_out/s4_emu_timeline.txt
