# Round 4, session 45: the emulated 8-rank C4 line after the in-batch planning change
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py --no-cpu-baseline --emulate-world 8 --config c4 --steps 30 --warmup 3 > gpurun_out/s45_c4_emu8.json 2> gpurun_out/s45_c4_emu8.err || { echo BENCH_FAIL; tail -5 gpurun_out/s45_c4_emu8.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/s45_c4_emu8.json')); print('c4_emu8', d['value'], d['ms_per_step'], [round(k.get('frac') or 0, 3) for k in d.get('kernels', [])])"
