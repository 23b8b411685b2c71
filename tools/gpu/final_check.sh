# round-end rehearsal: GPU tests, smoke(), default bench (with the CPU baseline) (developer script)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gt.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 600 python bench.py > gpurun_out/b_default.json 2> gpurun_out/b_default.err
