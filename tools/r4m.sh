# Round 4 (session 2i): the top-k bitonic sort on DPP / permlane exchanges
# instead of ds_bpermute — the evaluation tests, C2 A/B against the
# ds_bpermute build, the C5 line.
set -u
E=gpurun_out/r4m
mkdir -p $E
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread -k "evaluate or score_topk or topk or mf_c1 or users_rating or recall or metric" > $E/pytest_eval.log 2>&1
rc=$?; echo "pytest eval rc=$rc"; grep -E "passed|failed" $E/pytest_eval.log | tail -2; if [ $rc -ne 0 ]; then exit $rc; fi
for v in libmirec var_topk_bperm libmirec var_topk_bperm; do
  MIREC_LIB=$PWD/furusato_recommend_amd/$v.so timeout -k 10 300 python -u tools/eval_bench.py --reps 10 --dense 0 >> $E/eval_c2.jsonl 2> $E/eval_c2_$v.log
  rc=$?; echo "eval c2 $v rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
done
grep stream $E/eval_c2.jsonl | cut -c1-220; grep -c '"all_picks_ok": true' $E/eval_c2.jsonl
timeout -k 10 600 python -u tools/eval_bench.py --users 10000000 --items 1000000 --edges 200000000 --dim 256 --batch 10000 --reps 3 --dense 0 --check64 0 > $E/eval_c5.jsonl 2> $E/eval_c5.log
rc=$?; echo "eval c5 rc=$rc"; cut -c1-250 $E/eval_c5.jsonl
exit $rc
