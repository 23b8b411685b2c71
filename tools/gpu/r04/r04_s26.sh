# Round 4, session 26: PMC traffic passes for C4, C5 (tools/gpu/pmc_passes.sh) and C3 (pmc_c3.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/pmc_c4 BENCH_ARGS="--config c4" bash tools/gpu/pmc_passes.sh && echo c4 ok
OUT=gpurun_out/pmc_c5 BENCH_ARGS="--config c5" bash tools/gpu/pmc_passes.sh && echo c5 ok
OUT=gpurun_out/pmc_c3 bash tools/gpu/pmc_c3.sh && echo c3 ok
ls gpurun_out/pmc_c4 gpurun_out/pmc_c5 gpurun_out/pmc_c3
