# Round 4, session 5: host-side profile of the emulated 8-rank C2 step (cProfile), and the same
# bench without the profiler
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --no-cpu-baseline --emulate-world 8 --steps 100 --warmup 3 > gpurun_out/s5_emu.json 2> gpurun_out/s5_emu.err || { echo EMU_FAIL; tail -20 gpurun_out/s5_emu.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/s5_emu.json')); print('emu8', d['value'], d['ms_per_step'])"
timeout -k 10 300 python -u -m cProfile -o gpurun_out/s5_emu.prof bench.py --no-cpu-baseline --emulate-world 8 --steps 100 --warmup 3 > gpurun_out/s5_emu_prof.json 2> gpurun_out/s5_emu_prof.err || { echo PROF_FAIL; tail -20 gpurun_out/s5_emu_prof.err; exit 1; }
python3 -c "
import pstats
p = pstats.Stats('gpurun_out/s5_emu.prof'); p.sort_stats('tottime').print_stats(35)" > gpurun_out/s5_prof_tottime.txt
python3 -c "
import pstats
p = pstats.Stats('gpurun_out/s5_emu.prof'); p.sort_stats('cumulative').print_stats(45)" > gpurun_out/s5_prof_cum.txt
head -60 gpurun_out/s5_prof_tottime.txt
