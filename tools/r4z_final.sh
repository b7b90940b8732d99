# Round 4, last tree: the whole GPU suite, then the C3 line (fanout-mean
# changes) with its CPU baseline.
set -u
export TMPDIR=/tmp
E=gpurun_out/r4zf
mkdir -p $E
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 500 --timeout-method thread > $E/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $E/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/bench_sage.py --steps 20 > $E/bench_c3.log 2>&1 || { echo "c3 rc=$?"; exit 1; }
grep '^{' $E/bench_c3.log | cut -c1-200
