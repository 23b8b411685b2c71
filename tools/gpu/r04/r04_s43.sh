# Round 4, session 43: in-batch blocks per role (developer knob TTAMM_IB_BLOCKS; default 512) at
# C4, C2 in-batch and the C4 rank-of-8 kernel shape
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
b() {  # tag, env, args
  local tag=$1 pre=$2; shift 2
  env $pre timeout -k 10 400 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/s43_$tag.json 2> gpurun_out/s43_$tag.err || { echo BENCH_FAIL $tag; tail -5 gpurun_out/s43_$tag.err; return 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/s43_$tag.json')); print('$tag', d['value'], d['ms_per_step'])"
}
b c4 "" --config c4 && b c4_256 "TTAMM_IB_BLOCKS=256" --config c4 && b c4_1024 "TTAMM_IB_BLOCKS=1024" --config c4 \
  && b ib "" --negatives in-batch && b ib_256 "TTAMM_IB_BLOCKS=256" --negatives in-batch || exit 1
for n in 512 256 1024; do
  TTAMM_IB_BLOCKS=$n timeout -k 10 200 python -u tools/bench_inbatch.py --no-check > gpurun_out/s43_k$n.json 2> gpurun_out/s43_k$n.err || { echo K_FAIL; tail -5 gpurun_out/s43_k$n.err; exit 1; }
  echo "rank-of-8 kernel blocks=$n $(cat gpurun_out/s43_k$n.json)"
done
