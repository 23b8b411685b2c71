# the narrow weight gradients reduced on the aux stream beside the wide launch (new) vs build_old
# build_old: parity tests, alternating C2 A/B, and each library's kernels alone (--no-overlap) under rocprofv3
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "step_parity or deferred or optimizers or fullsize or sparse or clip or c1" > gpurun_out/s38_tests.log 2>&1
P=$GRAFT_REPO_ROOT/two-tower-augmented-with-adaptive-mimic-mechanism_amd
run() {  # name, lib
  TTAMM_LIBRARY=$2 timeout -k 10 200 python bench.py --no-cpu-baseline --no-exact-line --steps 20 --warmup 5 > gpurun_out/s38_$1.json 2> gpurun_out/s38_$1.err
  python -c "import json;d=json.loads(open('gpurun_out/s38_$1.json').read().strip().splitlines()[-1]);t=d['timeline'];print('$1',d['value'],d['ms_per_step'],t['ms_per_step_excl_closing_flush'],t['closing_flush_ms'])" >> gpurun_out/s38_ab.txt
}
for r in 1 2 3; do run old$r $P/build_old/libttamm.so; run new$r $P/ttamm/_native/libttamm.so; done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr38 -o run -- python3 bench.py --no-cpu-baseline --no-exact-line --steps 10 --warmup 3 > gpurun_out/s38_tr.json 2> gpurun_out/s38_tr.err
find gpurun_out/tr38 -name "*kernel_trace.csv" -exec cp {} gpurun_out/s38_tr.csv \;
rm -rf gpurun_out/tr38
