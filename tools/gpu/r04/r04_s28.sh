# Round 4, session 28: the aux stream restricted to a CU subset (bench.py --aux-cus) on the
# round-4 schedule, C2 and the emulated 8-rank C2
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for cus in 0 64 128 192 0; do
  for cfg in "" "--emulate-world 8 --steps 200 --warmup 5"; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --aux-cus $cus $cfg > gpurun_out/s28_x.json 2> gpurun_out/s28_x.err || { echo BENCH_FAIL $cus; tail -5 gpurun_out/s28_x.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/s28_x.json')); print('aux_cus=$cus [$cfg]', d['value'], d['ms_per_step'])"
  done
done
