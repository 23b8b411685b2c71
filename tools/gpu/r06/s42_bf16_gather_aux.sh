# bf16 towers: the ID-row gather on the aux stream right after the prologue (new) vs ahead of the first
# GEMM on the main stream (build_old): bf16 / sharded / full-size tests, alternating C5 A/B, C2 sanity
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "bf16 or c5 or sharded or fullsize or gate16 or step_parity" > gpurun_out/s42_tests.log 2>&1
P=$GRAFT_REPO_ROOT/two-tower-augmented-with-adaptive-mimic-mechanism_amd
run() {  # name, lib, args
  TTAMM_LIBRARY=$2 timeout -k 10 200 python bench.py --no-cpu-baseline --no-exact-line --steps 20 --warmup 5 $3 > gpurun_out/s42_$1.json 2> gpurun_out/s42_$1.err
  python -c "import json;d=json.loads(open('gpurun_out/s42_$1.json').read().strip().splitlines()[-1]);t=d['timeline'];print('$1',d['value'],d['ms_per_step'],t['ms_per_step_excl_closing_flush'],t['closing_flush_ms'])" >> gpurun_out/s42_ab.txt
}
for r in 1 2 3; do run c5old$r $P/build_old/libttamm.so "--config c5"; run c5new$r $P/ttamm/_native/libttamm.so "--config c5"; done
run c2new $P/ttamm/_native/libttamm.so ""
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr42 -o run -- python3 bench.py --no-cpu-baseline --no-exact-line --steps 10 --warmup 3 --config c5 > gpurun_out/s42_tr.json 2> gpurun_out/s42_tr.err
find gpurun_out/tr42 -name "*kernel_trace.csv" -exec cp {} gpurun_out/s42_tr.csv \;
rm -rf gpurun_out/tr42
