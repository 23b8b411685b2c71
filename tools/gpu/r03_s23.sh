# Round 3 session 23: gate outputs stored through per-wave LDS scratch as whole-row segments
# (default) vs from the MFMA layout (TTAMM_GATE_DIRECT_STORES=1): gate / step / sharded /
# autograd / full-size tests, bench A/B, kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_step_parity_gpu.py tests/test_kernels_gpu.py tests/test_golden_gpu.py tests/test_module_autograd_gpu.py tests/test_sharded_gpu.py tests/test_fullsize_parity_gpu.py tests/test_c1_gpu.py tests/test_category_gpu.py -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_s23.log 2>&1
rc=$?
tail -4 gpurun_out/gpu_tests_s23.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc"; exit $rc; fi
for v in slab direct slab direct; do
  if [ $v = direct ]; then export TTAMM_GATE_DIRECT_STORES=1; else unset TTAMM_GATE_DIRECT_STORES; fi
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/b_s23_$v.json 2> gpurun_out/b_s23_$v.err || { echo B_FAIL; tail -5 gpurun_out/b_s23_$v.err; exit 1; }
  python3 -c "
import json
d=json.load(open('gpurun_out/b_s23_$v.json')); print('$v', d['value'], d['ms_per_step'], d['final_loss'])"
done
unset TTAMM_GATE_DIRECT_STORES
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/stats -o run -- python3 bench.py --no-cpu-baseline > gpurun_out/stats_bench_s23.json 2> gpurun_out/stats_s23.err || { echo STATS_FAIL; exit 1; }
find gpurun_out/stats -name "*kernel_stats.csv" -exec cp {} gpurun_out/stats_kernel_stats_s23.csv \;
rm -rf gpurun_out/stats
grep gate gpurun_out/stats_kernel_stats_s23.csv | cut -c1-150
