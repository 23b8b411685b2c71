# Round 4, session 39: the closing measurement set on the final tree (split-K layer-1 forward for
# the in-batch steps) — smoke, the full GPU suite, the default C2 line (with the CPU baseline), its
# rocprofv3 kernel-trace --stats, C2 in-batch (2 and 3 splits), C4 (split, unsplit), C5, emulated
# 8-rank C4
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s39_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/s39_smoke.log; exit 1; }
tail -n 1 gpurun_out/s39_smoke.log
timeout -k 10 800 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/s39_tests.log 2>&1; rc=$?; grep -E "passed|failed|^FAILED|Error" gpurun_out/s39_tests.log | tail -8
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "suite rc=$rc"; exit $rc; fi
timeout -k 10 600 python -u bench.py > gpurun_out/s39_c2.json 2> gpurun_out/s39_c2.err || { echo BENCH_FAIL; tail -20 gpurun_out/s39_c2.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/s39_c2.json')); print('C2', d['value'], d['ms_per_step'], d['roofline'].get('frac'), d['cpu_baseline'])"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s39_prof -o run -- python3 bench.py --no-cpu-baseline > gpurun_out/s39_c2_prof.json 2> gpurun_out/s39_c2_prof.err || { echo PROF_FAIL; tail -20 gpurun_out/s39_c2_prof.err; exit 1; }
find gpurun_out/s39_prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/s39_c2_kernel_stats.csv \;
rm -rf gpurun_out/s39_prof
b() {  # tag, env, args
  local tag=$1 pre=$2; shift 2
  env $pre timeout -k 10 500 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/s39_$tag.json 2> gpurun_out/s39_$tag.err || { echo BENCH_FAIL $tag; tail -5 gpurun_out/s39_$tag.err; return 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/s39_$tag.json')); print('$tag', d['value'], d['ms_per_step'], [round(k.get('frac') or 0, 3) for k in d.get('kernels', [])])"
}
b inbatch "" --negatives in-batch && b inbatch_sp3 "TTAMM_GEMM_SPLITK_N=3" --negatives in-batch \
  && b c4 "" --config c4 && b c4_nosplit "TTAMM_GEMM_NO_SPLITK=1" --config c4 && b c5 "" --config c5 \
  && b c4_emu8 "" --emulate-world 8 --config c4 --steps 30 --warmup 3 || exit 1
