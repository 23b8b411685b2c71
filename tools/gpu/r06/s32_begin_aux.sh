# step count / AdamW constants published on the aux stream (prologue without its completion counter)
# + the register-scan sampler, vs build_old (HEAD before both): full GPU suite, then alternating A/B
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s32_gpu_tests.log 2>&1
P=$GRAFT_REPO_ROOT/two-tower-augmented-with-adaptive-mimic-mechanism_amd
run() {  # name, lib
  TTAMM_LIBRARY=$2 timeout -k 10 200 python bench.py --no-cpu-baseline --no-exact-line --steps 20 --warmup 5 > gpurun_out/s32_$1.json 2> gpurun_out/s32_$1.err
  python -c "import json;d=json.loads(open('gpurun_out/s32_$1.json').read().strip().splitlines()[-1]);t=d['timeline'];print('$1',d['value'],d['ms_per_step'],t['ms_per_step_excl_closing_flush'],t['closing_flush_ms'])" >> gpurun_out/s32_ab.txt
}
for r in 1 2 3; do run old$r $P/build_old/libttamm.so; run new$r $P/ttamm/_native/libttamm.so; done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr32 -o run -- python3 bench.py --no-cpu-baseline --no-exact-line --steps 10 --warmup 3 > gpurun_out/s32_tr.json 2> gpurun_out/s32_tr.err
find gpurun_out/tr32 -name "*kernel_trace.csv" -exec cp {} gpurun_out/s32_tr.csv \;
rm -rf gpurun_out/tr32
