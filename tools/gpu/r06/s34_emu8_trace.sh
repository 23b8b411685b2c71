# kernel trace of the emulated C2 rank of 8 (row-sharded step, MirrorComm)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr34 -o run -- python3 bench.py --no-cpu-baseline --no-exact-line --steps 10 --warmup 3 --emulate-world 8 > gpurun_out/s34_tr.json 2> gpurun_out/s34_tr.err
find gpurun_out/tr34 -name "*kernel_trace.csv" -exec cp {} gpurun_out/s34_tr.csv \;
rm -rf gpurun_out/tr34
