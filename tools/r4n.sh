# Round 4 (session 2j): the table-gradient pass 1 with v_readlane group
# broadcasts instead of ds_bpermute (84 VGPRs, six waves per SIMD) — tests,
# A/B against the __shfl build, kernel times, the C3 line.
set -u
E=gpurun_out/r4n
mkdir -p $E
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread -k "table_grad or sorted_leaf or c3_full_size or sage_training_steps or fused_table_adam or union_step or pipelined" > $E/pytest_tg.log 2>&1
rc=$?; echo "pytest tg rc=$rc"; grep -E "passed|failed" $E/pytest_tg.log | tail -2; if [ $rc -ne 0 ]; then exit $rc; fi
for v in libmirec var_tg_shfl libmirec var_tg_shfl; do
  MIREC_LIB=$PWD/furusato_recommend_amd/$v.so timeout -k 10 200 python -u tools/tg_bench.py >> $E/tg_bench.jsonl 2> $E/tg_bench_$v.log
  rc=$?; echo "tg_bench $v rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
done
cut -c1-200 $E/tg_bench.jsonl
for v in libmirec var_tg_shfl; do
  MIREC_LIB=$PWD/furusato_recommend_amd/$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $E/prof_$v -o run -- python3 tools/tg_bench.py --reps 20 > $E/prof_$v.log 2>&1
  rc=$?; echo "prof $v rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
done
find $E -name "*kernel_trace.csv" -delete
timeout -k 10 300 python -u tools/bench_sage.py --cpu-baseline 0 > $E/c3.json 2> $E/c3.log
rc=$?; echo "c3 rc=$rc"; cut -c1-200 $E/c3.json
exit $rc
