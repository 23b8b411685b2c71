# Round 4, session 33: every weight gradient on 128x96 tiles (TTAMM_WGRAD_ALL_NARROW=1) vs wide + narrow
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for pre in "" "TTAMM_WGRAD_ALL_NARROW=1" "" "TTAMM_WGRAD_ALL_NARROW=1"; do for cfg in "" "--config c4" "--config c5"; do
  env $pre timeout -k 10 400 python -u bench.py --no-cpu-baseline $cfg > gpurun_out/s33_x.json 2> gpurun_out/s33_x.err || { echo BENCH_FAIL $cfg; tail -5 gpurun_out/s33_x.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/s33_x.json')); print('[$pre] [$cfg]', d['value'], d['ms_per_step'])"
done; done
