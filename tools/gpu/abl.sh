set -e
cd $GRAFT_REPO_ROOT
for v in 0 1 2; do
  if [ $v = 0 ]; then export -n TTAMM_LIBRARY; unset TTAMM_LIBRARY; else export TTAMM_LIBRARY=$PWD/tools/gpu/libttamm_abl$v.so; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline --config c5 --steps 10 --warmup 3 > gpurun_out/abl_$v.json 2> gpurun_out/abl_$v.err
done
