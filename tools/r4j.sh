# Round 4 (session 2f): streamed top-k with occupancy-aware item chunking —
# its tests, C2 A/B against the fixed >= 1024-workgroup chunking, and the C5
# evaluation line (10 M users x 1 M items, d = 256: timing at 10 K users, the
# float64 near-tie check on 2 K users).
set -u
E=gpurun_out/r4j
mkdir -p $E
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread -k "evaluate or score_topk or topk or mf_c1 or users_rating" > $E/pytest_eval.log 2>&1
rc=$?; echo "pytest eval rc=$rc"; grep -E "passed|failed" $E/pytest_eval.log | tail -2; if [ $rc -ne 0 ]; then exit $rc; fi
for v in libmirec var_topk_fixed libmirec var_topk_fixed; do
  MIREC_LIB=$PWD/furusato_recommend_amd/$v.so timeout -k 10 300 python -u tools/eval_bench.py --reps 10 --dense 0 >> $E/eval_c2.jsonl 2> $E/eval_c2_$v.log
  rc=$?; echo "eval c2 $v rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
done
cut -c1-220 $E/eval_c2.jsonl
timeout -k 10 600 python -u tools/eval_bench.py --users 10000000 --items 1000000 --edges 200000000 --dim 256 --batch 10000 --reps 3 --dense 0 --check64 0 > $E/eval_c5.jsonl 2> $E/eval_c5.log
rc=$?; echo "eval c5 rc=$rc"; cut -c1-250 $E/eval_c5.jsonl; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u tools/eval_bench.py --users 10000000 --items 1000000 --edges 200000000 --dim 256 --batch 2000 --reps 1 --dense 0 --check64 1 > $E/eval_c5_check.jsonl 2> $E/eval_c5_check.log
rc=$?; echo "eval c5 check rc=$rc"; cut -c1-250 $E/eval_c5_check.jsonl
exit $rc
