# Round 4 (session 2b): the op_sel probe (full lines), the col_sums padding
# invariance test, table-gradient A/B (16-entry chunks) and kernel times at
# C3, the C3 profile, the C3 world-size projection.  rocprofv3 writes CSV and
# only the *_stats.csv files are kept (the merge-back limit is 64 MiB).
set -u
E=gpurun_out/r4f
mkdir -p $E
export TMPDIR=/tmp
REPS=30 timeout -k 10 300 python -u tools/op_sel_repro.py > $E/opsel.jsonl 2> $E/opsel.log
rc=$?; echo "opsel rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u -m pytest tests -m gpu -v -s --timeout 250 --timeout-method thread -k "col_sums" > $E/colsum.log 2>&1
rc=$?; echo "colsum rc=$rc"; grep -E "torch sum|passed|failed" $E/colsum.log | tail -8
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for v in libmirec var_tg_ch16 libmirec var_tg_ch16; do
  MIREC_LIB=$PWD/furusato_recommend_amd/$v.so timeout -k 10 200 python -u tools/tg_bench.py >> $E/tg_bench.jsonl 2> $E/tg_bench_$v.log
  rc=$?; echo "tg_bench $v rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
done
cat $E/tg_bench.jsonl
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $E/tgprof -o run -- python3 tools/tg_bench.py --reps 20 > $E/tgprof.log 2>&1
rc=$?; echo "tg prof rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $E/c3prof -o run -- python3 tools/bench_sage.py --steps 10 --warmup 3 --cpu-baseline 0 > $E/c3prof.log 2>&1
rc=$?; echo "c3 prof rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
find $E -type f ! -name "*.jsonl" ! -name "*.log" ! -name "*kernel_stats.csv" -delete
find $E -name "*kernel_stats.csv" | while read f; do echo "== $f"; grep -E "tg_" "$f" | cut -d, -f1-4 | cut -c1-170; done
timeout -k 10 600 python -u tools/bench_world_sim.py --model sage --worlds 1,2,8 --exchanges fetch --microbatches 1,2,4 --steps 10 > $E/world_sim_c3.jsonl 2> $E/world_sim_c3.log
rc=$?; echo "world sim rc=$rc"
du -sh $E
exit $rc
