# C2 bench line + steady-state kernel trace (developer script)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b_c2.json 2> gpurun_out/b_c2.err
timeout -k 10 300 python bench.py --no-cpu-baseline --config c5 > gpurun_out/b_c5.json 2> gpurun_out/b_c5.err
bash tools/gpu/trace_long.sh
