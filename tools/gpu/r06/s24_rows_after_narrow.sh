# the table-row updates after the narrow weight-gradient launch (TTAMM_ROWS_AFTER_NARROW builds) vs default
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=$GRAFT_REPO_ROOT/two-tower-augmented-with-adaptive-mimic-mechanism_amd
run() {  # name, library
  TTAMM_LIBRARY=$2 timeout -k 10 200 python bench.py --no-cpu-baseline --no-exact-line --steps 20 --warmup 5 > gpurun_out/s24_$1.json 2> gpurun_out/s24_$1.err
  python -c "import json;d=json.loads(open('gpurun_out/s24_$1.json').read().strip().splitlines()[-1]);t=d['timeline'];print('$1',d['value'],d['ms_per_step'],t['ms_per_step_excl_closing_flush'],t['closing_flush_ms'])" >> gpurun_out/s24_ran.txt
}
for r in 1 2 3; do
  run def$r $P/ttamm/_native/libttamm.so
  run v1_$r $P/build_ran1/libttamm.so
  run v2_$r $P/build_ran2/libttamm.so
done
for v in 1 2; do
TTAMM_LIBRARY=$P/build_ran$v/libttamm.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr_v$v -o run -- python3 bench.py --no-cpu-baseline --no-exact-line --steps 10 --warmup 3 > gpurun_out/s24_tr_v$v.json 2> gpurun_out/s24_tr_v$v.err
find gpurun_out/tr_v$v -name "*kernel_trace.csv" -exec cp {} gpurun_out/s24_tr_v$v.csv \;
rm -rf gpurun_out/tr_v$v
done
