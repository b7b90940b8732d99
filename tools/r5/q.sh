# Round 5 (q): streamed top-k A/B vs HEAD (tkh) at C2 — evaluation tests first;
# then C5-like
# d = 256 (the D > 128 path) with its float64 check.
set -u
export TMPDIR=/tmp
E=gpurun_out/r5q
mkdir -p $E
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 500 --timeout-method thread -k "evaluat or topk or recall" > $E/pytest_eval.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $E/pytest_eval.log
[ $rc = 0 ] || exit $rc
for rep in 1 2; do
  for L in tkh prod; do
    if [ $L = prod ]; then unset MIREC_LIB; else export MIREC_LIB=var/libmirec_$L.so; fi
    timeout -k 10 300 python -u tools/eval_bench.py --reps 10 --dense 0 --check64 $([ $rep = 1 ] && echo 1 || echo 0) >> $E/eval_ab.jsonl 2>> $E/eval_ab.log || { echo "eval_bench $L failed"; tail $E/eval_ab.log; exit 1; }
  done
done
unset MIREC_LIB
cut -c1-200 $E/eval_ab.jsonl
timeout -k 10 600 python -u tools/eval_bench.py --users 2000000 --items 1000000 --edges 40000000 --dim 256 --batch 2000 --reps 3 --dense 0 > $E/eval_d256.log 2>&1 || { echo "eval rc=$?"; tail $E/eval_d256.log; exit 1; }
grep '^{' $E/eval_d256.log | cut -c1-250
