# row_update / piece_sum with the segment bounds and first row loaded one round trip earlier (new) vs
# build_old: parity tests, alternating C2 A/B, and each library's kernels alone (--no-overlap) under rocprofv3
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "step_parity or deferred or optimizers or fullsize or sparse or padding or sharded" > gpurun_out/s37_tests.log 2>&1
P=$GRAFT_REPO_ROOT/two-tower-augmented-with-adaptive-mimic-mechanism_amd
run() {  # name, lib
  TTAMM_LIBRARY=$2 timeout -k 10 200 python bench.py --no-cpu-baseline --no-exact-line --steps 20 --warmup 5 > gpurun_out/s37_$1.json 2> gpurun_out/s37_$1.err
  python -c "import json;d=json.loads(open('gpurun_out/s37_$1.json').read().strip().splitlines()[-1]);t=d['timeline'];print('$1',d['value'],d['ms_per_step'],t['ms_per_step_excl_closing_flush'],t['closing_flush_ms'])" >> gpurun_out/s37_ab.txt
}
for r in 1 2 3; do run old$r $P/build_old/libttamm.so; run new$r $P/ttamm/_native/libttamm.so; done
for v in old new; do
  L=$P/ttamm/_native/libttamm.so; [ $v = old ] && L=$P/build_old/libttamm.so
  TTAMM_LIBRARY=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p37$v -o run -- python3 bench.py --no-cpu-baseline --no-exact-line --steps 20 --warmup 5 --no-overlap > gpurun_out/s37_noovl_$v.json 2> gpurun_out/s37_noovl_$v.err
  find gpurun_out/p37$v -name "*kernel_stats.csv" -exec cp {} gpurun_out/s37_noovl_${v}_stats.csv \;
  rm -rf gpurun_out/p37$v
done
