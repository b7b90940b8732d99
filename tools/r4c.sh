# Round 4 final tree: the whole GPU suite, smoke, the C2 bench line (with the
# oracle parity leg), C2 rocprof passes, C3 / C4 lines and stats, the C3
# world simulation with the pipelined exchange, the C2 / C5 evaluation lines.
# Every GPU step has its own time limit; a failure ends the script.
set -u
export TMPDIR=/tmp
E=gpurun_out/r4c
mkdir -p $E
timeout -k 10 1500 python -u -m pytest tests -m gpu -q -rf --timeout 600 --timeout-method thread > $E/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 $E/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $E/smoke.log 2>&1 || { echo "smoke rc=$?"; exit 1; }
tail -2 $E/smoke.log
timeout -k 10 700 python bench.py > $E/bench_c2.log 2>&1 || { echo "bench rc=$?"; tail -5 $E/bench_c2.log; exit 1; }
grep '^{' $E/bench_c2.log | cut -c1-300
PROF_OUT=$E/prof bash tools/profile.sh || exit 1
timeout -k 10 400 python tools/bench_sage.py --steps 20 > $E/bench_c3.log 2>&1 || { echo "c3 rc=$?"; exit 1; }
grep '^{' $E/bench_c3.log | cut -c1-200
timeout -k 10 400 python tools/bench_sasrec.py --steps 100 > $E/bench_c4.log 2>&1 || { echo "c4 rc=$?"; exit 1; }
grep '^{' $E/bench_c4.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $E/c4 -o run --output-format csv -- python3 tools/bench_sasrec.py --steps 10 --warmup 3 --cpu-baseline 0 > $E/c4.log 2>&1 || { echo "c4 trace rc=$?"; exit 1; }
timeout -k 10 600 python tools/bench_world_sim.py --model sage --worlds 1,2,8 --exchanges fetch,routed --microbatches 1,2,4 --steps 10 > $E/world_sim_c3.jsonl 2>&1 || { echo "world sim rc=$?"; exit 1; }
grep '^{' $E/world_sim_c3.jsonl | cut -c1-250
echo "r4c ok"
