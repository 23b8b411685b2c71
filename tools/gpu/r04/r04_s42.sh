# Round 4, session 42: the generic gate's output pass as gate_mix_kernel (rows.hip) after an
# EPI_STORE GEMM — smoke, the full GPU suite, then C5 / C4 with and without it
# (TTAMM_GATE_OUT_EPILOGUE=1 = the fused epilogue), C2
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s42_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/s42_smoke.log; exit 1; }
tail -n 1 gpurun_out/s42_smoke.log
timeout -k 10 800 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/s42_tests.log 2>&1; rc=$?; grep -E "passed|failed|^FAILED|Error" gpurun_out/s42_tests.log | tail -8
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "suite rc=$rc"; exit $rc; fi
b() {  # tag, env, args
  local tag=$1 pre=$2; shift 2
  env $pre timeout -k 10 500 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/s42_$tag.json 2> gpurun_out/s42_$tag.err || { echo BENCH_FAIL $tag; tail -5 gpurun_out/s42_$tag.err; return 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/s42_$tag.json')); print('$tag', d['value'], d['ms_per_step'])"
}
b c5 "" --config c5 && b c5_epi "TTAMM_GATE_OUT_EPILOGUE=1" --config c5 && b c4 "" --config c4 \
  && b c4_epi "TTAMM_GATE_OUT_EPILOGUE=1" --config c4 && b c5b "" --config c5 && b c2 "" || exit 1
