# the remaining bench lines of the round (c4 with the bulk gather, emulated ranks of 8, in-batch) and
# the rocprofv3 kernel stats of the driver's command
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in "c4:--config c4" "c4w8:--config c4 --emulate-world 8 --no-gather-bulk" "c2w8:--emulate-world 8" "c2ib:--negatives in-batch"; do
  n=${cfg%%:*}; a=${cfg#*:}
  timeout -k 10 400 python bench.py --no-cpu-baseline --steps 20 --warmup 5 $a > gpurun_out/s30_$n.json 2> gpurun_out/s30_$n.err
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof30 -o run -- python3 bench.py --no-cpu-baseline --no-exact-line --steps 20 --warmup 5 > gpurun_out/s30_prof_bench.json 2> gpurun_out/s30_prof.err
find gpurun_out/prof30 -name "*kernel_stats.csv" -exec cp {} gpurun_out/s30_c2_kernel_stats.csv \;
find gpurun_out/prof30 -name "*kernel_trace.csv" -exec cp {} gpurun_out/s30_c2_kernel_trace.csv \;
rm -rf gpurun_out/prof30
