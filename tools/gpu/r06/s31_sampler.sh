# sampler: short positive lists scanned from registers (new) vs binary search (build_old); sampler tests
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "sampl or smoke or step_parity" > gpurun_out/s31_tests.log 2>&1
P=$GRAFT_REPO_ROOT/two-tower-augmented-with-adaptive-mimic-mechanism_amd
run() {  # name, lib
  TTAMM_LIBRARY=$2 timeout -k 10 200 python bench.py --no-cpu-baseline --no-exact-line --steps 20 --warmup 5 > gpurun_out/s31_$1.json 2> gpurun_out/s31_$1.err
  python -c "import json;d=json.loads(open('gpurun_out/s31_$1.json').read().strip().splitlines()[-1]);t=d['timeline'];print('$1',d['value'],d['ms_per_step'],t['ms_per_step_excl_closing_flush'],t['closing_flush_ms'])" >> gpurun_out/s31_ab.txt
}
for r in 1 2 3; do run old$r $P/build_old/libttamm.so; run new$r $P/ttamm/_native/libttamm.so; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof31 -o run -- python3 bench.py --no-cpu-baseline --no-exact-line --steps 20 --warmup 5 > gpurun_out/s31_prof_bench.json 2> gpurun_out/s31_prof.err
find gpurun_out/prof31 -name "*kernel_stats.csv" -exec cp {} gpurun_out/s31_kernel_stats.csv \;
rm -rf gpurun_out/prof31
