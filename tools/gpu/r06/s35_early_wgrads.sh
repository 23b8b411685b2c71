# early (narrow) weight gradients: 0 = main stream between dgrad and wide (HEAD), 1 = aux stream ahead
# of the row updates, 2 = a side stream (new default); step parity tests, alternating A/B, a trace
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "step_parity or deferred or smoke or optimizers or fullsize" > gpurun_out/s35_tests.log 2>&1
P=$GRAFT_REPO_ROOT/two-tower-augmented-with-adaptive-mimic-mechanism_amd
run() {  # name, lib
  TTAMM_LIBRARY=$2 timeout -k 10 200 python bench.py --no-cpu-baseline --no-exact-line --steps 20 --warmup 5 > gpurun_out/s35_$1.json 2> gpurun_out/s35_$1.err
  python -c "import json;d=json.loads(open('gpurun_out/s35_$1.json').read().strip().splitlines()[-1]);t=d['timeline'];print('$1',d['value'],d['ms_per_step'],t['ms_per_step_excl_closing_flush'],t['closing_flush_ms'])" >> gpurun_out/s35_ab.txt
}
for r in 1 2 3; do run e0_$r $P/build_e0/libttamm.so; run e1_$r $P/build_e1/libttamm.so; run e2_$r $P/ttamm/_native/libttamm.so; done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr35 -o run -- python3 bench.py --no-cpu-baseline --no-exact-line --steps 10 --warmup 3 > gpurun_out/s35_tr.json 2> gpurun_out/s35_tr.err
find gpurun_out/tr35 -name "*kernel_trace.csv" -exec cp {} gpurun_out/s35_tr.csv \;
rm -rf gpurun_out/tr35
