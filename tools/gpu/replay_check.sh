set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_deferred_gpu.py tests/test_fullsize_gpu.py tests/test_c1_gpu.py > gpurun_out/replay.log 2>&1
for cfg in c2 c4 c5; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --config $cfg > gpurun_out/rp_${cfg}.json 2> gpurun_out/rp.err
done
