# weight-gradient rows per split per class in the C2 step (developer library, TTAMM_WGRAD_RPS<class>)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
DEV=$GRAFT_REPO_ROOT/two-tower-augmented-with-adaptive-mimic-mechanism_amd/build_devrun/libttamm.so
run() {  # name, env
  env TTAMM_LIBRARY=$DEV $2 timeout -k 10 200 python bench.py --no-cpu-baseline --no-exact-line --steps 20 --warmup 5 > gpurun_out/s27_$1.json 2> gpurun_out/s27_$1.err
  python -c "import json;d=json.loads(open('gpurun_out/s27_$1.json').read().strip().splitlines()[-1]);t=d['timeline'];print('$1',d['value'],d['ms_per_step'],t['ms_per_step_excl_closing_flush'],t['closing_flush_ms'])" >> gpurun_out/s27_rps.txt
}
for r in 1 2; do
  run def$r "X=1"
  for v in 256 320 448 512 640; do run n${v}_$r "TTAMM_WGRAD_RPS0=$v"; done
  for v in 448 704 832; do run w${v}_$r "TTAMM_WGRAD_RPS1=$v"; done
done
