#!/bin/bash
# Final-tree evidence (round 3): full GPU suite + smoke, C2 bench line (CPU
# baseline + Recall@20 leg), C3 / C4 lines with CPU baselines, C3 / C4
# rocprof kernel stats, GEMM shapes.  Each GPU step has its own limit and a
# failure ends the script.
set -u
export TMPDIR=/tmp
E=gpurun_out/r3c
mkdir -p $E
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread > $E/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $E/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $E/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -5 $E/smoke.log; exit 1; }
tail -1 $E/smoke.log
timeout -k 10 600 python bench.py > $E/bench_c2.log 2>&1 || { echo "bench rc=$?"; tail -5 $E/bench_c2.log; exit 1; }
grep '^{' $E/bench_c2.log | cut -c1-200
timeout -k 10 300 python tools/bench_sage.py --steps 20 > $E/bench_c3.log 2>&1 || { echo "c3 rc=$?"; exit 1; }
grep '^{' $E/bench_c3.log | cut -c1-160
timeout -k 10 300 python tools/bench_sasrec.py --steps 100 > $E/bench_c4.log 2>&1 || { echo "c4 rc=$?"; exit 1; }
grep '^{' $E/bench_c4.log | cut -c1-160
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $E/c3 -o run --output-format csv -- python3 tools/bench_sage.py --steps 10 --warmup 3 --cpu-baseline 0 > $E/c3.log 2>&1 || { echo "c3 trace rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $E/c4 -o run --output-format csv -- python3 tools/bench_sasrec.py --steps 10 --warmup 3 --cpu-baseline 0 > $E/c4.log 2>&1 || { echo "c4 trace rc=$?"; exit 1; }
timeout -k 10 200 python tools/gemm_bench.py > $E/gemm.jsonl 2> $E/gemm.err || { echo "gemm rc=$?"; exit 1; }
echo "evidence ok"
