# four-register-set ring for the 128 x 128 weight-gradient tiles: r0 = two sets (HEAD), r4 = ring on
# the bf16 32-k tiles, r44 = ring on the fp32 16-k tiles too; C5 (bf16) and C4 (fp32) lines, alternating
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=$GRAFT_REPO_ROOT/two-tower-augmented-with-adaptive-mimic-mechanism_amd
run() {  # name, lib, args
  TTAMM_LIBRARY=$P/build_$2/libttamm.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-exact-line --steps 20 --warmup 5 $3 > gpurun_out/s28_$1.json 2> gpurun_out/s28_$1.err
  python -c "
import json;d=json.loads(open('gpurun_out/s28_$1.json').read().strip().splitlines()[-1]);t=d['timeline']
w=[k for k in d['kernels'] if k['kernel'].startswith('wide')] if 'kernels' in d else []
print('$1',d['value'],d['ms_per_step'],t['ms_per_step_excl_closing_flush'],[k.get('avg_launch_ms') for k in w])" >> gpurun_out/s28_ring.txt
}
for r in 1 2; do
  for v in r0 r4 r44; do run c5_${v}_$r $v "--config c5"; done
  for v in r0 r44; do run c4_${v}_$r $v "--config c4 --no-gather-bulk"; done
done
