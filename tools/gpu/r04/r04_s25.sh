# Round 4, session 25: PMC traffic passes (tools/gpu/pmc_passes.sh) for C2 and C2 in-batch
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/pmc_c2 BENCH_ARGS="" bash tools/gpu/pmc_passes.sh && echo c2 ok
OUT=gpurun_out/pmc_c2ib BENCH_ARGS="--negatives in-batch" bash tools/gpu/pmc_passes.sh && echo c2ib ok
ls gpurun_out/pmc_c2 gpurun_out/pmc_c2ib
