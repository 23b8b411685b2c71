# bench's per-kernel event pairs vs none, alternating (C2, the driver's K / W)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2 3; do
  for ev in every-step none; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-exact-line --steps 20 --warmup 5 --kernel-events $ev > gpurun_out/s22_$ev$r.json 2> gpurun_out/s22_$ev$r.err
    python -c "import json,sys;d=json.loads(open('gpurun_out/s22_$ev$r.json').read().strip().splitlines()[-1]);print('$ev$r',d['value'],d['ms_per_step'],d['timeline'])" >> gpurun_out/s22_events.txt
  done
done
