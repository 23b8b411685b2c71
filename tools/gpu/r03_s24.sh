# Round 3 session 24: weight-gradient split-K rows per split at C5 (bf16 towers; its wide launch
# fetched 5x its algorithmic bytes in the final PMC pass) — default model vs fixed values
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in default 128 256 512 1024; do
  if [ $v = default ]; then unset TTAMM_WGRAD_ROWS_PER_SPLIT; else export TTAMM_WGRAD_ROWS_PER_SPLIT=$v; fi
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --config c5 --steps 100 --warmup 3 > gpurun_out/b_s24_$v.json 2> gpurun_out/b_s24_$v.err || { echo B_FAIL; tail -5 gpurun_out/b_s24_$v.err; exit 1; }
  python3 -c "
import json
d=json.load(open('gpurun_out/b_s24_$v.json')); ks=[(k['kernel'][:30], k.get('avg_launch_ms')) for k in d['kernels'] if 'avg_launch_ms' in k]; print('$v', d['value'], d['ms_per_step'], ks)"
done
