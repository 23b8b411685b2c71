# FETCH_SIZE / WRITE_SIZE passes + a bench line (developer script)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
run_pass() {
    local name=$1; shift
    timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/pmc_$name -o run -- python3 bench.py --no-cpu-baseline --steps 40 --warmup 3 $BENCH_ARGS > gpurun_out/pmc_${name}_bench.json 2> gpurun_out/pmc_${name}.err
    find gpurun_out/pmc_$name -name "*counter_collection.csv" -exec cp {} gpurun_out/pmc_${name}.csv \;
    rm -rf gpurun_out/pmc_$name
}
run_pass fetch FETCH_SIZE
run_pass write WRITE_SIZE
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b_c2.json 2> gpurun_out/b_c2.err
