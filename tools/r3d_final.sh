#!/bin/bash
# Final-tree check: full GPU suite, smoke, C4 / C3 lines.
set -u
export TMPDIR=/tmp
E=gpurun_out/r3d
mkdir -p $E
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread > $E/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $E/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $E/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -5 $E/smoke.log; exit 1; }
tail -1 $E/smoke.log
timeout -k 10 300 python tools/bench_sasrec.py --steps 100 > $E/bench_c4.log 2>&1 || { echo "c4 rc=$?"; exit 1; }
grep '^{' $E/bench_c4.log | cut -c1-160
timeout -k 10 300 python tools/bench_sage.py --steps 20 > $E/bench_c3.log 2>&1 || { echo "c3 rc=$?"; exit 1; }
grep '^{' $E/bench_c3.log | cut -c1-160
echo "final ok"
