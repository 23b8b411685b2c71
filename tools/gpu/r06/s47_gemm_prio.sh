# gemm_x_kernel waves at s_setprio 2 (build_p2) vs default priority: alternating C2 / C5 A/B
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=$GRAFT_REPO_ROOT/two-tower-augmented-with-adaptive-mimic-mechanism_amd
run() {  # name, lib, args
  TTAMM_LIBRARY=$2 timeout -k 10 200 python bench.py --no-cpu-baseline --no-exact-line --steps 20 --warmup 5 $3 > gpurun_out/s47_$1.json 2> gpurun_out/s47_$1.err
  python -c "import json;d=json.loads(open('gpurun_out/s47_$1.json').read().strip().splitlines()[-1]);t=d['timeline'];print('$1',d['value'],d['ms_per_step'],t['ms_per_step_excl_closing_flush'],t['closing_flush_ms'])" >> gpurun_out/s47_ab.txt
}
for r in 1 2 3; do run def$r $P/ttamm/_native/libttamm.so ""; run p2_$r $P/build_p2/libttamm.so ""; done
for r in 1 2; do run c5def$r $P/ttamm/_native/libttamm.so "--config c5"; run c5p2_$r $P/build_p2/libttamm.so "--config c5"; done
