set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for n in 32 64 128 200; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --replay-slices $n > gpurun_out/sl_$n.json 2> gpurun_out/sl.err
done
for n in 32 128; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --config c4 --replay-slices $n > gpurun_out/sl4_$n.json 2> gpurun_out/sl.err
done
