set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in c4 c2 c5; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --config $cfg > gpurun_out/sc_${cfg}_aux.json 2> gpurun_out/sc.err
  TTAMM_SLICE_MAIN=1 timeout -k 10 300 python bench.py --no-cpu-baseline --config $cfg > gpurun_out/sc_${cfg}_main.json 2> gpurun_out/sc.err
done
