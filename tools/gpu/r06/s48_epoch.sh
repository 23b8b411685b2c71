# the shipped binary: python bench.py with no arguments (one C2 epoch + the closing flush, CPU baseline, exact sub-line)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/s48_epoch.json 2> gpurun_out/s48_epoch.err
