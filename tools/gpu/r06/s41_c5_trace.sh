# kernel trace of the C5 step (bf16 towers) on the final tree
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr41 -o run -- python3 bench.py --no-cpu-baseline --no-exact-line --steps 10 --warmup 3 --config c5 > gpurun_out/s41_tr.json 2> gpurun_out/s41_tr.err
find gpurun_out/tr41 -name "*kernel_trace.csv" -exec cp {} gpurun_out/s41_tr.csv \;
rm -rf gpurun_out/tr41
