# split-bf16 GEMM ablations at the C2 shapes + one SQ counter pass over the micro-benchmark
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
B=two-tower-augmented-with-adaptive-mimic-mechanism_amd/build
timeout -k 10 120 $B/gemm_bench > gpurun_out/gemm_base.txt 2>&1 || { echo BASE_FAIL; cat gpurun_out/gemm_base.txt; exit 1; }
timeout -k 10 120 $B/gemm_bench_xabl3 > gpurun_out/gemm_xabl3.txt 2>&1 || { echo ABL3_FAIL; exit 1; }
timeout -k 10 120 $B/gemm_bench_xabl2 > gpurun_out/gemm_xabl2.txt 2>&1 || { echo ABL2_FAIL; exit 1; }
cat gpurun_out/gemm_base.txt gpurun_out/gemm_xabl3.txt gpurun_out/gemm_xabl2.txt
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/pmc_gemm -o run -- $B/gemm_bench > gpurun_out/pmc_gemm.txt 2>&1 || { echo PMC_FAIL; tail -5 gpurun_out/pmc_gemm.txt; exit 1; }
find gpurun_out/pmc_gemm -name "*counter_collection.csv" -exec cp {} gpurun_out/pmc_gemm_sq.csv \;
rm -rf gpurun_out/pmc_gemm
echo done
