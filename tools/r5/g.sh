# Round 5 (g): streamed top-k A/B at C2 — committed form (tkc), simplified
# filter (tks), product (filter of tile j-1 interleaved with tile j's MFMA
# chain); the product's evaluation tests first.
set -u
export TMPDIR=/tmp
E=gpurun_out/r5g
mkdir -p $E
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 500 --timeout-method thread -k "evaluat or topk or recall" > $E/pytest_eval.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -12 $E/pytest_eval.log
[ $rc = 0 ] || exit $rc
for rep in 1 2; do
  for L in tkc tks prod; do
    if [ $L = prod ]; then unset MIREC_LIB; else export MIREC_LIB=var/libmirec_$L.so; fi
    echo "== $L" >> $E/eval_ab.log
    timeout -k 10 300 python -u tools/eval_bench.py --reps 10 --dense 0 --check64 $([ $rep = 1 ] && echo 1 || echo 0) >> $E/eval_ab.jsonl 2>> $E/eval_ab.log || { echo "eval_bench $L failed"; tail $E/eval_ab.log; exit 1; }
  done
done
cut -c1-250 $E/eval_ab.jsonl
