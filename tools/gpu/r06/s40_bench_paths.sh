# bench.py after the HipTimingEvent shutdown guard: the driver's command and a 2-rank (gloo, one GPU) run
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/s40_driver.json 2> gpurun_out/s40_driver.err
timeout -k 10 400 python bench.py --gpus 2 --dist-backend gloo --steps 5 --warmup 2 --no-cpu-baseline --no-exact-line > gpurun_out/s40_w2.json 2> gpurun_out/s40_w2.err
