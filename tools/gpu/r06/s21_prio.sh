set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python tools/diag/prio_probe.py --rounds 3 > gpurun_out/s21_prio.txt 2>&1
