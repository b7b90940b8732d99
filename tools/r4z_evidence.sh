# Round 4 final tree, part 2 (PART=1: the C2 bench line (oracle parity leg),
# C2 rocprof passes, C3 / C4 lines; PART=2: C3 / C4 kernel stats, FETCH / WRITE of
# the run-aligned table-gradient sum, the C3 world simulation.  rocprofv3
# writes CSV; only the *_stats.csv and counter CSVs of the kept passes stay.
set -u
export TMPDIR=/tmp
E=gpurun_out/r4z
mkdir -p $E
PART=${PART:-1}
if [ "$PART" = 1 ]; then
timeout -k 10 700 python bench.py > $E/bench_c2.log 2>&1 || { echo "bench rc=$?"; tail -5 $E/bench_c2.log; exit 1; }
grep '^{' $E/bench_c2.log | cut -c1-400
PROF_OUT=$E/prof bash tools/profile.sh || exit 1
find $E/prof -name "*kernel_trace.csv" -delete
timeout -k 10 400 python tools/bench_sage.py --steps 20 > $E/bench_c3.log 2>&1 || { echo "c3 rc=$?"; exit 1; }
grep '^{' $E/bench_c3.log | cut -c1-300
timeout -k 10 400 python tools/bench_sasrec.py --steps 100 > $E/bench_c4.log 2>&1 || { echo "c4 rc=$?"; exit 1; }
grep '^{' $E/bench_c4.log | cut -c1-300
echo "r4z part 1 ok"
exit 0
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $E/c3 -o run --output-format csv -- python3 tools/bench_sage.py --steps 10 --warmup 3 --cpu-baseline 0 > $E/c3prof.log 2>&1 || { echo "c3 trace rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $E/c4 -o run --output-format csv -- python3 tools/bench_sasrec.py --steps 10 --warmup 3 --cpu-baseline 0 > $E/c4prof.log 2>&1 || { echo "c4 trace rc=$?"; exit 1; }
find $E/c3 $E/c4 -name "*kernel_trace.csv" -delete
timeout -k 10 200 python -u tools/tg_sum_bytes.py > $E/tg_counts.json 2> $E/tg_counts.log || { echo "tg counts rc=$?"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex tg_sum -d $E/tgf -o run --output-format csv -- python3 tools/bench_sage.py --steps 5 --warmup 2 --cpu-baseline 0 > $E/tgf.log 2>&1 || { echo "pmc fetch rc=$?"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex tg_sum -d $E/tgw -o run --output-format csv -- python3 tools/bench_sage.py --steps 5 --warmup 2 --cpu-baseline 0 > $E/tgw.log 2>&1 || { echo "pmc write rc=$?"; exit 1; }
python tools/tg_sum_bytes.py --counts $E/tg_counts.json --fetch $E/tgf --write $E/tgw --out $E/pmc_tg_sum.json | grep counter_over
find $E/tgf $E/tgw -name "*kernel_trace.csv" -delete
timeout -k 10 600 python -u tools/bench_world_sim.py --model sage --worlds 1,2,8 --exchanges fetch,routed --microbatches 1,2,4 --steps 10 > $E/world_sim_c3.jsonl 2> $E/world_sim_c3.log || { echo "world sim rc=$?"; exit 1; }
du -sh $E
echo "r4z ok"
