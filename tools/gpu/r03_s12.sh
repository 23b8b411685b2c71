# Round 3 session 12: VALU issue rates of the replay's instructions; SQ counters of the default
# bench (per kernel); steady-state kernel trace for the step timeline
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
B=two-tower-augmented-with-adaptive-mimic-mechanism_amd/build
timeout -k 10 120 $B/valu_bench > gpurun_out/valu_bench.txt 2>&1 || { echo VB_FAIL; cat gpurun_out/valu_bench.txt; exit 1; }
cat gpurun_out/valu_bench.txt
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/pmc_step -o run -- python3 bench.py --no-cpu-baseline --steps 40 --warmup 3 > gpurun_out/pmc_step.txt 2>&1 || { echo PMC_FAIL; tail -5 gpurun_out/pmc_step.txt; exit 1; }
find gpurun_out/pmc_step -name "*counter_collection.csv" -exec cp {} gpurun_out/pmc_step_sq.csv \;
rm -rf gpurun_out/pmc_step
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS --output-format csv -d gpurun_out/pmc_step2 -o run -- python3 bench.py --no-cpu-baseline --steps 40 --warmup 3 > gpurun_out/pmc_step2.txt 2>&1 || { echo PMC2_FAIL; tail -5 gpurun_out/pmc_step2.txt; exit 1; }
find gpurun_out/pmc_step2 -name "*counter_collection.csv" -exec cp {} gpurun_out/pmc_step2_sq.csv \;
rm -rf gpurun_out/pmc_step2
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_l -o run -- python3 bench.py --no-cpu-baseline --steps 120 --warmup 3 > gpurun_out/trace_l_bench.json 2> gpurun_out/trace_l.err || { echo TRACE_FAIL; exit 1; }
find gpurun_out/trace_l -name "*kernel_trace.csv" -exec cp {} gpurun_out/trace_l_kernels.csv \;
rm -rf gpurun_out/trace_l
python3 tools/trace_timeline.py gpurun_out/trace_l_kernels.csv > gpurun_out/timeline_s12.txt && head -80 gpurun_out/timeline_s12.txt
