# Round 4 (session 1b): split score tiles in the streamed top-k (tests,
# x6 vs f32 at C2 with the float64 near-tie check, C5 line), tg_sum
# counter bytes at C3, the C4 line with back-to-back attention timing.
set -u
mkdir -p gpurun_out/r4b
export TMPDIR=/tmp
# PART=1: the op_sel probe, the C4 oracle test, the eval tests and lines;
# PART=2: tg_sum counters, C3 profile, C4 line, the torch-colsum rerun.
PART=${PART:-1}
if [ "$PART" = 1 ]; then
REPS=50 timeout -k 10 200 python -u tools/op_sel_repro.py > gpurun_out/r4b/opsel.jsonl 2> gpurun_out/r4b/opsel.log
rc=$?; echo "opsel rc=$rc"; cat gpurun_out/r4b/opsel.jsonl
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u -m pytest tests -m gpu -v -s --timeout 500 --timeout-method thread -k "c4_batch_step" > gpurun_out/r4b/pytest_c4.log 2>&1
rc=$?; echo "pytest c4 rc=$rc"; tail -4 gpurun_out/r4b/pytest_c4.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "evaluate or score_topk or mf_c1 or topk or trajectory or distinct_rows or union_step or routed or repeatable or pipelined" > gpurun_out/r4b/pytest_eval.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/r4b/pytest_eval.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for v in libmirec var_topk_f32; do
  MIREC_LIB=$PWD/furusato_recommend_amd/$v.so timeout -k 10 300 python -u tools/eval_bench.py --reps 10 > gpurun_out/r4b/eval_c2_$v.jsonl 2>&1
  rc=$?; echo "eval $v rc=$rc"; cat gpurun_out/r4b/eval_c2_$v.jsonl
  if [ $rc -ne 0 ]; then exit $rc; fi
done
exit 0
fi
REPS=30 timeout -k 10 300 python -u tools/op_sel_repro.py > gpurun_out/r4b/opsel2.jsonl 2> gpurun_out/r4b/opsel2.log
rc=$?; echo "opsel2 rc=$rc"; cat gpurun_out/r4b/opsel2.jsonl
if [ $rc -ne 0 ]; then exit $rc; fi
for v in libmirec var_tg_head var_tg_ch4; do
  MIREC_LIB=$PWD/furusato_recommend_amd/$v.so timeout -k 10 200 python -u tools/tg_bench.py >> gpurun_out/r4b/tg_bench.jsonl 2> gpurun_out/r4b/tg_bench_$v.log
  rc=$?; echo "tg_bench $v rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
done
cat gpurun_out/r4b/tg_bench.jsonl
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r4b/tgprof -o run -- python3 tools/tg_bench.py --reps 20 > gpurun_out/r4b/tgprof.log 2>&1
rc=$?; echo "tg prof rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/tg_sum_bytes.py > gpurun_out/r4b/tg_counts.json 2> gpurun_out/r4b/tg_counts.log
rc=$?; echo "tg counts rc=$rc"; cat gpurun_out/r4b/tg_counts.json
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex tg_sum -d gpurun_out/r4b/tgf -o run --output-format csv -- python3 tools/bench_sage.py --steps 5 --warmup 2 --cpu-baseline 0 > gpurun_out/r4b/tgf.log 2>&1
rc=$?; echo "pmc fetch rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex tg_sum -d gpurun_out/r4b/tgw -o run --output-format csv -- python3 tools/bench_sage.py --steps 5 --warmup 2 --cpu-baseline 0 > gpurun_out/r4b/tgw.log 2>&1
rc=$?; echo "pmc write rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
python tools/tg_sum_bytes.py --counts gpurun_out/r4b/tg_counts.json --fetch gpurun_out/r4b/tgf --write gpurun_out/r4b/tgw --out gpurun_out/r4b/pmc_tg_sum.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4b/c3prof -o run -- python3 tools/bench_sage.py --steps 10 --warmup 3 --cpu-baseline 0 > gpurun_out/r4b/c3prof.log 2>&1
rc=$?; echo "c3 prof rc=$rc"; tail -1 gpurun_out/r4b/c3prof.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python -u tools/bench_sasrec.py > gpurun_out/r4b/c4.json 2> gpurun_out/r4b/c4.log
rc=$?; echo "c4 rc=$rc"; cat gpurun_out/r4b/c4.json
if [ $rc -ne 0 ]; then exit $rc; fi
# the round-3 form of the captured DP step (torch sum(0) for the bias
# gradients): its captured-vs-eager test, once
MIREC_TORCH_COLSUM=1 timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 500 --timeout-method thread -k "captured_step_equals_eager" > gpurun_out/r4b/torch_colsum.log 2>&1
rc=$?; echo "torch colsum rc=$rc"; tail -3 gpurun_out/r4b/torch_colsum.log
exit 0
