# Round 5 (f): the whole GPU suite on the current tree, then the streamed
# evaluation at C5's d = 256 (the top-k's D > 128 path) with its float64 check.
set -u
export TMPDIR=/tmp
E=gpurun_out/r5f
mkdir -p $E
timeout -k 10 1100 python -u -m pytest tests -m gpu -q -rf --timeout 500 --timeout-method thread > $E/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 $E/pytest.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u tools/eval_bench.py --users 2000000 --items 1000000 --edges 40000000 --dim 256 --batch 2000 --reps 3 --dense 0 > $E/eval_d256.log 2>&1 || { echo "eval rc=$?"; tail $E/eval_d256.log; exit 1; }
grep '^{' $E/eval_d256.log | cut -c1-300
exit $rc
