# Round 4, session 24: rocprofv3 --kernel-trace --stats (csv) of the default C2 bench command
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s24_prof -o run -- python3 bench.py --no-cpu-baseline > gpurun_out/s24_c2_prof.json 2> gpurun_out/s24_c2_prof.err || { echo PROF_FAIL; tail -20 gpurun_out/s24_c2_prof.err; exit 1; }
find gpurun_out/s24_prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/s24_c2_kernel_stats.csv \;
rm -rf gpurun_out/s24_prof
head -n 8 gpurun_out/s24_c2_kernel_stats.csv | cut -c1-200
python3 -c "import json; d=json.load(open('gpurun_out/s24_c2_prof.json')); print('C2 under rocprof', d['value'], d['ms_per_step'], d['roofline']['ms_per_step'])"
