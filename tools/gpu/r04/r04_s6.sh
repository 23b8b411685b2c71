# Round 4, session 6: the pipelined in-batch kernel vs the split kernel, its parity tests
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in x p; do
  for pos in 65536 8192; do
    TTAMM_IB_KERNEL=$v timeout -k 10 120 python -u tools/bench_inbatch.py --positives $pos > gpurun_out/s6_ib_${v}_$pos.json 2> gpurun_out/s6_ib_${v}_$pos.err || { echo IB_FAIL $v $pos; tail -20 gpurun_out/s6_ib_${v}_$pos.err; exit 1; }
    echo $v $pos; cat gpurun_out/s6_ib_${v}_$pos.json
  done
done
TTAMM_IB_KERNEL=p timeout -k 10 600 python -u -m pytest tests/test_inbatch_op_gpu.py tests/test_inbatch_gpu.py -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/s6_ib_tests.log 2>&1; tail -3 gpurun_out/s6_ib_tests.log
