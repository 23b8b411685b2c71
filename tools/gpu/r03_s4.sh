# Round 3 session 4: new sharded-option and module-autograd tests, then PMC passes (C2 all
# three groups; C4/C5 fetch+write) and the kernel-trace --stats summary of the default bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_sharded_options_gpu.py tests/test_module_autograd_gpu.py -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_new.log 2>&1
rc=$?
tail -30 gpurun_out/gpu_tests_new.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
bash tools/gpu/pmc_passes.sh || { echo PMC_C2_FAIL; exit 1; }
for c in c4 c5; do
  for p in fetch:FETCH_SIZE write:WRITE_SIZE; do
    n=${p%%:*}; k=${p##*:}
    timeout -s KILL 240 rocprofv3 --pmc $k --output-format csv -d gpurun_out/pmc_${c}_$n -o run -- python3 bench.py --no-cpu-baseline --steps 40 --warmup 3 --config $c > gpurun_out/pmc_${c}_${n}_bench.json 2> gpurun_out/pmc_${c}_${n}.err || { echo PMC_${c}_FAIL; exit 1; }
    find gpurun_out/pmc_${c}_$n -name "*counter_collection.csv" -exec cp {} gpurun_out/pmc_${c}_${n}.csv \;
    rm -rf gpurun_out/pmc_${c}_$n
  done
done
echo "pytest rc=$rc"
