# rocprofv3 PMC passes (one counter group per run, as MI355X_MICROARCH.md prescribes) and the
# kernel-trace --stats summary of the bench command; outputs copied to gpurun_out/pmc_* .
# Developer script: BENCH_ARGS selects the config, OUT the output directory (default gpurun_out).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${OUT:-gpurun_out}
mkdir -p $O
run_pass() {  # name, counters...
    local name=$1; shift
    timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d $O/pmc_$name -o run -- python3 bench.py --no-cpu-baseline --no-exact-line --steps 40 --warmup 3 $BENCH_ARGS > $O/pmc_${name}_bench.json 2> $O/pmc_${name}.err
    find $O/pmc_$name -name "*counter_collection.csv" -exec cp {} $O/pmc_${name}.csv \;
    rm -rf $O/pmc_$name
}
run_pass fetch FETCH_SIZE
run_pass write WRITE_SIZE
run_pass valu SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_WAVES SQ_INSTS_SALU
timeout -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 bench.py --no-cpu-baseline --no-exact-line $BENCH_ARGS > $O/stats_bench.json 2> $O/stats.err
find $O/stats -name "*kernel_stats.csv" -exec cp {} $O/stats_kernel_stats.csv \;
rm -rf $O/stats
