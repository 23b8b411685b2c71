# rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; one run each) of the C3 retrieval bench
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${OUT:-gpurun_out}
mkdir -p $O
for c in FETCH_SIZE WRITE_SIZE; do
  n=$(echo $c | cut -d_ -f1 | tr A-Z a-z)
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $O/pmc_c3_$n -o run -- python3 tools/bench_retrieval.py --reps 2 --cpu-queries 0 > $O/pmc_c3_${n}_bench.json 2> $O/pmc_c3_$n.err
  find $O/pmc_c3_$n -name "*counter_collection.csv" -exec cp {} $O/pmc_c3_$n.csv \;
  rm -rf $O/pmc_c3_$n
done
