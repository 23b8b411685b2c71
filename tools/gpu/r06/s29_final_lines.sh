# bench --kernel-events roofline (new default) vs every-step; then the round's bench lines and the
# rocprofv3 kernel stats of the driver command
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
ab() {  # name, args
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-exact-line --steps 20 --warmup 5 $2 > gpurun_out/s29_$1.json 2> gpurun_out/s29_$1.err
  python -c "import json;d=json.loads(open('gpurun_out/s29_$1.json').read().strip().splitlines()[-1]);t=d['timeline'];print('$1',d['value'],d['ms_per_step'],t['ms_per_step_excl_closing_flush'],t['closing_flush_ms'],d['roofline']['ms_per_step'],[k.get('avg_launch_ms') for k in d['kernels']])" >> gpurun_out/s29_ab.txt
}
for r in 1 2 3; do ab roof$r "--kernel-events roofline"; ab every$r "--kernel-events every-step"; done
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/s29_driver.json 2> gpurun_out/s29_driver.err
for cfg in "c5:--config c5" "c4:--config c4" "c4w8:--config c4 --emulate-world 8 --no-gather-bulk" "c2w8:--emulate-world 8" "c2ib:--negatives in-batch"; do
  n=${cfg%%:*}; a=${cfg#*:}
  timeout -k 10 400 python bench.py --no-cpu-baseline --steps 20 --warmup 5 $a > gpurun_out/s29_$n.json 2> gpurun_out/s29_$n.err
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof29 -o run -- python3 bench.py --no-cpu-baseline --no-exact-line --steps 20 --warmup 5 > gpurun_out/s29_prof_bench.json 2> gpurun_out/s29_prof.err
find gpurun_out/prof29 -name "*kernel_stats.csv" -exec cp {} gpurun_out/s29_c2_kernel_stats.csv \;
find gpurun_out/prof29 -name "*kernel_trace.csv" -exec cp {} gpurun_out/s29_c2_kernel_trace.csv \;
rm -rf gpurun_out/prof29
