# Round 4, session 41: SQ counters of the C5 step's bf16 GEMM chain (one PMC pass, 8 SQ counters),
# evidence for the next round's C5 work (is the wide weight-gradient launch waiting on memory?)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD --output-format csv -d gpurun_out/pmc_c5sq -o run -- python3 bench.py --config c5 --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/s41_bench.json 2> gpurun_out/s41.err || { echo PMC_FAIL; tail -5 gpurun_out/s41.err; exit 1; }
find gpurun_out/pmc_c5sq -name "*counter_collection.csv" -exec cp {} gpurun_out/s41_c5_sq.csv \;
rm -rf gpurun_out/pmc_c5sq
python3 tools/pmc_kernel.py gpurun_out/s41_c5_sq.csv --match gemm > gpurun_out/s41_c5_sq.json && head -c 1500 gpurun_out/s41_c5_sq.json
