# Round 3 session 18: rolling-slice count sweep at C2 (shorter lags move replay work from the
# catch-up before the gate, on the critical path, to the slice overlapping the backward)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for n in 64 32 16 24 48 64; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --replay-slices $n > gpurun_out/b_s18_$n.json 2> gpurun_out/b_s18_$n.err || { echo B_FAIL; tail -5 gpurun_out/b_s18_$n.err; exit 1; }
  python3 -c "
import json
d=json.load(open('gpurun_out/b_s18_$n.json')); r=d['roofline']; print('$n', d['value'], d['ms_per_step'], r['ms_per_step'], r.get('parts_ms_per_step'), d['timeline'])"
done
