# Round 3 final, part B: the PMC passes of the default bench (FETCH_SIZE, WRITE_SIZE, VALU by
# type) and of the C5 and C4 benches, each with its kernel stats (summarised here afterwards by
# tools/pmc_summary.py into profiles/pmc_traffic.json)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/pmc_c2 bash tools/gpu/pmc_passes.sh || { echo PMC_FAIL; exit 1; }
OUT=gpurun_out/pmc_c5 BENCH_ARGS="--config c5" bash tools/gpu/pmc_passes.sh || { echo PMC_C5_FAIL; exit 1; }
OUT=gpurun_out/pmc_c4 BENCH_ARGS="--config c4" bash tools/gpu/pmc_passes.sh || { echo PMC_C4_FAIL; exit 1; }
ls -la gpurun_out/pmc_c2 gpurun_out/pmc_c5 gpurun_out/pmc_c4
