# Round 4 (session 2d): the table-gradient pass 1 with the owned run's
# extension rows in flight beside the chunk's rows + 11-bit sort passes:
# its tests, A/B times and kernel times at C3, the C3 line.
set -u
E=gpurun_out/r4h
mkdir -p $E
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread -k "table_grad or sorted_leaf or c3_full_size or sage_training_steps or fused_table_adam or union_step or pipelined" > $E/pytest_tg.log 2>&1
rc=$?; echo "pytest tg rc=$rc"; grep -E "passed|failed|Error" $E/pytest_tg.log | tail -3
if [ $rc -ne 0 ]; then exit $rc; fi
for v in libmirec var_tg_seqext var_tg_head libmirec var_tg_seqext; do
  MIREC_LIB=$PWD/furusato_recommend_amd/$v.so timeout -k 10 200 python -u tools/tg_bench.py >> $E/tg_bench.jsonl 2> $E/tg_bench_$v.log
  rc=$?; echo "tg_bench $v rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
done
cut -c1-200 $E/tg_bench.jsonl
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $E/tgprof -o run -- python3 tools/tg_bench.py --reps 20 > $E/tgprof.log 2>&1
rc=$?; echo "tg prof rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
find $E -name "*kernel_trace.csv" -delete
find $E -name "*kernel_stats.csv" | while read f; do grep -E "tg_|trampoline" "$f" | cut -d, -f1-4 | sed 's/(.*"//' | cut -c1-120; done
timeout -k 10 300 python -u tools/bench_sage.py > $E/c3.json 2> $E/c3.log
rc=$?; echo "c3 rc=$rc"; cut -c1-300 $E/c3.json
exit $rc
