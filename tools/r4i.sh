# Round 4 (session 2e): table-gradient A/B at C3 — libmirec (run-aligned,
# extension rows beside the chunk's, window indices beside its keys, 11-bit
# sort), var_tg_seq11 (run-aligned, extension after the chunk, window
# indices beside its keys, 11-bit sort), var_tg_old11 (chunk partials of
# round 3 + 11-bit sort), var_tg_head (round 3's as is).  Results equal
# within each family (hash).  Then the kernel times of the fastest two.
set -u
E=gpurun_out/r4i
mkdir -p $E
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -v -x --timeout 250 --timeout-method thread -k "table_grad" > $E/pytest_tg.log 2>&1
rc=$?; echo "pytest tg rc=$rc"; grep -E "passed|failed" $E/pytest_tg.log | tail -2; if [ $rc -ne 0 ]; then exit $rc; fi
for v in libmirec var_tg_seq11 var_tg_old11 var_tg_head libmirec var_tg_seq11 var_tg_old11 var_tg_head; do
  MIREC_LIB=$PWD/furusato_recommend_amd/$v.so timeout -k 10 200 python -u tools/tg_bench.py >> $E/tg_bench.jsonl 2> $E/tg_bench_$v.log
  rc=$?; echo "tg_bench $v rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
done
cut -c1-120 $E/tg_bench.jsonl
for v in libmirec var_tg_seq11 var_tg_old11; do
  MIREC_LIB=$PWD/furusato_recommend_amd/$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $E/prof_$v -o run -- python3 tools/tg_bench.py --reps 20 > $E/prof_$v.log 2>&1
  rc=$?; echo "prof $v rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
done
find $E -name "*kernel_trace.csv" -delete
for v in libmirec var_tg_seq11 var_tg_old11; do echo "== $v"; find $E/prof_$v -name "*kernel_stats.csv" | while read f; do grep -E "tg_sum|tg_fixup" "$f" | cut -d, -f1-4 | sed 's/(.*"//' ; done; done
