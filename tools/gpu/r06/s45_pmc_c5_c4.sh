# PMC passes of C5 and C4 on the shipped binary (tools/gpu/pmc_passes.sh per config)
set -e
cd $GRAFT_REPO_ROOT
BENCH_ARGS="--config c5" OUT=gpurun_out/c5 bash tools/gpu/pmc_passes.sh
BENCH_ARGS="--config c4 --no-gather-bulk" OUT=gpurun_out/c4 bash tools/gpu/pmc_passes.sh
