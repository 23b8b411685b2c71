# Round 3 session 14: split-bf16 GEMM ablations at the C2 shapes (hh-only MFMA, no k-loop
# traffic), VALU instruction-type counters of the default bench (replay issue-cycle roofline)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
B=two-tower-augmented-with-adaptive-mimic-mechanism_amd/build
timeout -k 10 120 $B/gemm_bench > gpurun_out/gemm_base.txt 2>&1 || { echo BASE_FAIL; cat gpurun_out/gemm_base.txt; exit 1; }
timeout -k 10 120 $B/gemm_bench_xabl2 > gpurun_out/gemm_xabl2.txt 2>&1 || { echo ABL2_FAIL; exit 1; }
timeout -k 10 120 $B/gemm_bench_xabl3 > gpurun_out/gemm_xabl3.txt 2>&1 || { echo ABL3_FAIL; exit 1; }
grep -E "split" gpurun_out/gemm_base.txt gpurun_out/gemm_xabl2.txt gpurun_out/gemm_xabl3.txt | grep -v fp64
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_SALU SQ_WAVES SQ_INSTS_LDS --output-format csv -d gpurun_out/pmc_valu -o run -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/pmc_valu.txt 2>&1 || { echo PMC_FAIL; tail -5 gpurun_out/pmc_valu.txt; exit 1; }
find gpurun_out/pmc_valu -name "*counter_collection.csv" -exec cp {} gpurun_out/pmc_valu.csv \;
rm -rf gpurun_out/pmc_valu
echo done
