# rocprofv3 kernel stats of short bench runs of the given configs (developer script)
# usage: bash tools/gpu/stats_cfg.sh c5 c4 ...
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in "$@"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/st_$cfg -o run -- python3 bench.py --no-cpu-baseline --config $cfg --steps 30 --warmup 3 > gpurun_out/st_${cfg}_bench.json 2> gpurun_out/st_${cfg}.err
  find gpurun_out/st_$cfg -name "*kernel_stats.csv" -exec cp {} gpurun_out/st_${cfg}_kernel_stats.csv \;
  rm -rf gpurun_out/st_$cfg
done
