#!/bin/bash
# Round-end evidence on one GPU box: C2 rocprofv3 passes (kernel stats +
# FETCH_SIZE + WRITE_SIZE), the C2 bench line, C3 / C4 bench lines with their
# CPU baselines and kernel stats.  Every GPU step has its own time limit and a
# failure ends the script.
set -u
export TMPDIR=/tmp
E=gpurun_out/ev
mkdir -p $E
PROF_OUT=$E/prof2 bash tools/profile.sh || exit 1
timeout -k 10 600 python bench.py > $E/bench_c2.log 2>&1 || { echo "bench rc=$?"; exit 1; }
grep '^{' $E/bench_c2.log | cut -c1-200
timeout -k 10 300 python tools/bench_sage.py --steps 20 > $E/bench_c3.log 2>&1 || { echo "c3 rc=$?"; exit 1; }
grep '^{' $E/bench_c3.log | cut -c1-200
timeout -k 10 300 python tools/bench_sasrec.py --steps 100 > $E/bench_c4.log 2>&1 || { echo "c4 rc=$?"; exit 1; }
grep '^{' $E/bench_c4.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $E/c3 -o run --output-format csv -- python3 tools/bench_sage.py --steps 10 --warmup 3 --cpu-baseline 0 > $E/c3.log 2>&1 || { echo "c3 trace rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $E/c4 -o run --output-format csv -- python3 tools/bench_sasrec.py --steps 10 --warmup 3 --cpu-baseline 0 > $E/c4.log 2>&1 || { echo "c4 trace rc=$?"; exit 1; }

# skewed C2 graph (Zipf item popularity): bench line and kernel stats
timeout -k 10 300 python bench.py --kind zipf --steps 20 --warmup 3 --cpu-baseline off --quality-steps 0 --parity 0 > $E/bench_c2_zipf.log 2>&1 || { echo "zipf rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $E/zipf -o run --output-format csv -- python3 bench.py --kind zipf --steps 10 --warmup 3 --cpu-baseline off --quality-steps 0 --parity 0 > $E/zipf.log 2>&1 || { echo "zipf trace rc=$?"; exit 1; }
echo "zipf ok"
echo "evidence ok"
