# Round 4, last tree (after the DP exchange and table-Adam changes): the whole
# GPU suite, the C2 bench line (oracle parity + CPU baseline) and its rocprof
# passes, the C3 / C4 lines, the C3 / C4 kernel stats.  CSV output; trace CSVs
# deleted so only the stats stay.
set -u
export TMPDIR=/tmp
E=gpurun_out/r4last
mkdir -p $E
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 500 --timeout-method thread > $E/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $E/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 700 python bench.py > $E/bench_c2.log 2>&1 || { echo "bench rc=$?"; tail -5 $E/bench_c2.log; exit 1; }
grep '^{' $E/bench_c2.log | cut -c1-300
PROF_OUT=$E/prof bash tools/profile.sh || exit 1
find $E/prof -name "*kernel_trace.csv" -delete
timeout -k 10 400 python tools/bench_sage.py --steps 20 > $E/bench_c3.log 2>&1 || { echo "c3 rc=$?"; exit 1; }
grep '^{' $E/bench_c3.log | cut -c1-200
timeout -k 10 400 python tools/bench_sasrec.py --steps 100 > $E/bench_c4.log 2>&1 || { echo "c4 rc=$?"; exit 1; }
grep '^{' $E/bench_c4.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $E/c3 -o run --output-format csv -- python3 tools/bench_sage.py --steps 10 --warmup 3 --cpu-baseline 0 > $E/c3prof.log 2>&1 || { echo "c3 trace rc=$?"; exit 1; }
find $E/c3 -name "*kernel_trace.csv" -delete
du -sh $E
echo "r4last ok"
