# round-6 session 3: HEAD baseline — driver's bench command, then kernel traces with and without the aux stream
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/s20_bench.json 2> gpurun_out/s20_bench.err
for mode in ovl noovl; do
  args=""; [ $mode = noovl ] && args="--no-overlap"
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr_$mode -o run -- python3 bench.py --no-cpu-baseline --no-exact-line --steps 10 --warmup 3 $args > gpurun_out/s20_tr_$mode.json 2> gpurun_out/s20_tr_$mode.err
  find gpurun_out/tr_$mode -name "*kernel_trace.csv" -exec cp {} gpurun_out/s20_tr_$mode.csv \;
  rm -rf gpurun_out/tr_$mode
done
