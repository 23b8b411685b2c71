# Round 4, session 27: knob sweep on the round-4 schedule (C2 default bench): weight-gradient rows
# per split, replay constants in scalar registers, slice placement
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for combo in "" "TTAMM_WGRAD_ROWS_PER_SPLIT=256" "TTAMM_WGRAD_ROWS_PER_SPLIT=512" "TTAMM_WGRAD_ROWS_PER_SPLIT=1024" "TTAMM_REPLAY_SCALAR=1" "TTAMM_SLICE_MAIN=1" "TTAMM_SLICE_LATE=1" ""; do
  env $combo timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/s27_x.json 2> gpurun_out/s27_x.err || { echo BENCH_FAIL "$combo"; tail -5 gpurun_out/s27_x.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/s27_x.json')); print('[$combo]', d['value'], d['ms_per_step'])"
done
