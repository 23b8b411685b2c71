# PMC passes of the C2 in-batch line and the emulated ranks of 8 on the shipped binary
set -e
cd $GRAFT_REPO_ROOT
BENCH_ARGS="--negatives in-batch" OUT=gpurun_out/c2_inbatch bash tools/gpu/pmc_passes.sh
BENCH_ARGS="--emulate-world 8" OUT=gpurun_out/c2_w8 bash tools/gpu/pmc_passes.sh
BENCH_ARGS="--config c4 --emulate-world 8 --no-gather-bulk" OUT=gpurun_out/c4_w8 bash tools/gpu/pmc_passes.sh
