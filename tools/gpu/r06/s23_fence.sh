# device-scope sync / timing events vs system-scope (the HEAD library = build_old), alternating
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
OLD=$GRAFT_REPO_ROOT/two-tower-augmented-with-adaptive-mimic-mechanism_amd/build_old/libttamm_old.so
run() {  # name, env, args
  env $2 timeout -k 10 200 python bench.py --no-cpu-baseline --no-exact-line --steps 20 --warmup 5 $3 > gpurun_out/s23_$1.json 2> gpurun_out/s23_$1.err
  python -c "import json;d=json.loads(open('gpurun_out/s23_$1.json').read().strip().splitlines()[-1]);t=d['timeline'];print('$1',d['value'],d['ms_per_step'],t['ms_per_step_excl_closing_flush'],t['closing_flush_ms'],d['roofline']['ms_per_step'])" >> gpurun_out/s23_fence.txt
}
for r in 1 2 3; do
  run old_torch$r "TTAMM_LIBRARY=$OLD" "--event-kind torch"
  run new_device$r "X=1" "--event-kind device"
  run new_torch$r "X=1" "--event-kind torch"
  run new_none$r "X=1" "--kernel-events none"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr_new -o run -- python3 bench.py --no-cpu-baseline --no-exact-line --steps 10 --warmup 3 > gpurun_out/s23_tr_new.json 2> gpurun_out/s23_tr_new.err
find gpurun_out/tr_new -name "*kernel_trace.csv" -exec cp {} gpurun_out/s23_tr_new.csv \;
rm -rf gpurun_out/tr_new
