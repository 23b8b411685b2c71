# Round 4, session 3: in-batch kernel variants (4 waves x 2 blocks, 8 waves double-buffered) at the
# C4 rank shape, SQ counters of the 4-wave kernel, the SGD tests
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for w in 4 8; do
  TTAMM_IB_WAVES=$w timeout -k 10 120 python -u tools/bench_inbatch.py > gpurun_out/s3_ib_w$w.json 2> gpurun_out/s3_ib_w$w.err || { echo IB_FAIL $w; tail -20 gpurun_out/s3_ib_w$w.err; exit 1; }
  cat gpurun_out/s3_ib_w$w.json
done
TTAMM_IB_WAVES=4 timeout -k 10 120 python -u tools/bench_inbatch.py --batch 8192 --positives 8192 > gpurun_out/s3_ib_c2_w4.json 2>&1 && cat gpurun_out/s3_ib_c2_w4.json
TTAMM_IB_WAVES=8 timeout -k 10 120 python -u tools/bench_inbatch.py --batch 8192 --positives 8192 > gpurun_out/s3_ib_c2_w8.json 2>&1 && cat gpurun_out/s3_ib_c2_w8.json
pass() {
  local name=$1; shift
  TTAMM_IB_WAVES=4 timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/pmc_$name -o run -- python3 tools/bench_inbatch.py --no-check --reps 3 > gpurun_out/pmc_$name.out 2>&1 || { echo PMC_FAIL $name; tail -5 gpurun_out/pmc_$name.out; return 1; }
  find gpurun_out/pmc_$name -name "*counter_collection.csv" -exec cp {} gpurun_out/s3_pmc_$name.csv \;
  rm -rf gpurun_out/pmc_$name
}
pass sq1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS && \
pass sq2 SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD && \
python3 tools/pmc_kernel.py gpurun_out/s3_pmc_sq1.csv gpurun_out/s3_pmc_sq2.csv --match inbatch_x > gpurun_out/s3_pmc_ib.json; cat gpurun_out/s3_pmc_ib.json
timeout -k 10 600 python -u -m pytest tests/test_optimizers_gpu.py -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/s3_opt.log 2>&1; tail -5 gpurun_out/s3_opt.log
