# the first layer's weight pad inside the (now shorter) step prologue: TTAMM_PROLOGUE_PREP=1 (developer library) vs off
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
DEV=$GRAFT_REPO_ROOT/two-tower-augmented-with-adaptive-mimic-mechanism_amd/build_devrun/libttamm.so
run() {  # name, env
  env TTAMM_LIBRARY=$DEV $2 timeout -k 10 200 python bench.py --no-cpu-baseline --no-exact-line --steps 20 --warmup 5 > gpurun_out/s33_$1.json 2> gpurun_out/s33_$1.err
  python -c "import json;d=json.loads(open('gpurun_out/s33_$1.json').read().strip().splitlines()[-1]);t=d['timeline'];print('$1',d['value'],d['ms_per_step'],t['ms_per_step_excl_closing_flush'],t['closing_flush_ms'])" >> gpurun_out/s33_ab.txt
}
for r in 1 2 3; do run off$r "X=1"; run prep$r "TTAMM_PROLOGUE_PREP=1"; done
