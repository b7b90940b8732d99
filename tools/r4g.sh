# Round 4 (session 2c): the run-aligned table-gradient sum — its tests first
# (every run length / alignment, hub rows, float64, repeatability, the C3
# sorted-vs-atomic and bitwise-repeatable steps), then A/B times against the
# previous kernel and per-kernel times at C3; the op_sel probe (full lines);
# the col_sums padding test; the C2 bench line (bpr / finalize kernels now
# built without packed-f32 ops); the C3 world-size projection.
set -u
E=gpurun_out/r4g
mkdir -p $E
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread -k "table_grad or sorted_leaf or c3_full_size or sage_training_steps or fused_table_adam or union_step or pipelined or col_sums" > $E/pytest_tg.log 2>&1
rc=$?; echo "pytest tg rc=$rc"; grep -E "passed|failed|Error" $E/pytest_tg.log | tail -5
if [ $rc -ne 0 ]; then exit $rc; fi
grep "torch sum" $E/pytest_tg.log | head -4
for v in libmirec var_tg_head var_tg_ch16 var_tg_sort11 libmirec var_tg_head var_tg_sort11; do
  MIREC_LIB=$PWD/furusato_recommend_amd/$v.so timeout -k 10 200 python -u tools/tg_bench.py >> $E/tg_bench.jsonl 2> $E/tg_bench_$v.log
  rc=$?; echo "tg_bench $v rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
done
cut -c1-200 $E/tg_bench.jsonl
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $E/tgprof -o run -- python3 tools/tg_bench.py --reps 20 > $E/tgprof.log 2>&1
rc=$?; echo "tg prof rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
find $E -type f ! -name "*.jsonl" ! -name "*.log" ! -name "*kernel_stats.csv" -delete
find $E -name "*kernel_stats.csv" | while read f; do grep -E "tg_|onesweep" "$f" | cut -d, -f1-4 | sed 's/rocprim.*onesweep/onesweep/' | cut -c1-150; done
# attention backward with phase A's P / dS kept in LDS (MIREC_ATTN_PDS=1)
MIREC_LIB=$PWD/furusato_recommend_amd/var_attn_pds.so timeout -k 10 300 python -u -m pytest tests -m gpu -v -x --timeout 250 --timeout-method thread -k "attention or attn" > $E/pytest_attn_pds.log 2>&1
rc=$?; echo "pytest attn pds rc=$rc"; grep -E "passed|failed" $E/pytest_attn_pds.log | tail -2
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for v in libmirec var_attn_pds; do
  MIREC_LIB=$PWD/furusato_recommend_amd/$v.so timeout -k 10 200 python -u tools/attn_bench.py --mixes c4 --batches 2048 --reps 20 > $E/attn_$v.jsonl 2> $E/attn_$v.log
  rc=$?; echo "attn bench $v rc=$rc"; grep -i "bwd\|packed" $E/attn_$v.jsonl | cut -c1-250; if [ $rc -ne 0 ]; then exit $rc; fi
done
REPS=30 timeout -k 10 300 python -u tools/op_sel_repro.py > $E/opsel.jsonl 2> $E/opsel.log
rc=$?; echo "opsel rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py > $E/bench_c2.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $E/bench_c2.log | cut -c1-600; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/bench_sage.py > $E/c3.json 2> $E/c3.log
rc=$?; echo "c3 rc=$rc"; cut -c1-400 $E/c3.json; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 500 python -u tools/bench_world_sim.py --model sage --worlds 1,2,8 --exchanges fetch --microbatches 1,2,4 --steps 10 > $E/world_sim_c3.jsonl 2> $E/world_sim_c3.log
rc=$?; echo "world sim rc=$rc"
du -sh $E
exit $rc
