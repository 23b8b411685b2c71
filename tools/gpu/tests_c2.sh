set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gt.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b_c2.json 2> gpurun_out/b_c2.err
bash tools/gpu/trace_long.sh
