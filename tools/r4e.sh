# Round 4 (session 2): the op_sel probe with MFMA and non-MFMA waves sharing
# every SIMD, the captured DP test with torch's sum(0) (the round-3 form),
# the table-gradient kernels' times at C3, the C3 profile, the C3 world-size
# projection with the pipelined exchange.  Trace CSVs are deleted after the
# stats are kept (the merge-back limit).
set -u
E=gpurun_out/r4e
mkdir -p $E
export TMPDIR=/tmp
REPS=30 timeout -k 10 300 python -u tools/op_sel_repro.py > $E/opsel3.jsonl 2> $E/opsel3.log
rc=$?; echo "opsel3 rc=$rc"; cut -c1-400 $E/opsel3.jsonl
if [ $rc -ne 0 ]; then exit $rc; fi
MIREC_TORCH_COLSUM=1 timeout -k 10 300 python -u -m pytest tests -m gpu -v -x --timeout 250 --timeout-method thread -k "captured_step_equals_eager and routed" > $E/torch_colsum.log 2>&1
rc=$?; echo "torch colsum rc=$rc"; grep -E "Error|assert|passed|failed" $E/torch_colsum.log | cut -c1-300 | tail -12
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $E/tgprof -o run -- python3 tools/tg_bench.py --reps 20 > $E/tgprof.log 2>&1
rc=$?; echo "tg prof rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $E/c3prof -o run -- python3 tools/bench_sage.py --steps 10 --warmup 3 --cpu-baseline 0 > $E/c3prof.log 2>&1
rc=$?; echo "c3 prof rc=$rc"; tail -1 $E/c3prof.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi
find $E -name "*kernel_trace.csv" -delete
find $E -name "*kernel_stats.csv" | while read f; do echo "== $f"; grep -E "tg_|Name" "$f" | cut -d, -f1-5 | cut -c1-160; done
timeout -k 10 600 python -u tools/bench_world_sim.py --model sage --worlds 1,2,8 --exchanges fetch,routed --microbatches 1,2,4 --steps 10 > $E/world_sim_c3.jsonl 2> $E/world_sim_c3.log
rc=$?; echo "world sim rc=$rc"; grep '^{' $E/world_sim_c3.jsonl | cut -c1-300
du -sh $E
exit $rc
