# Round 3 evidence, part 2: C2 rocprofv3 passes (kernel stats + FETCH_SIZE +
# WRITE_SIZE), C3 / C4 lines with BASELINE §3 CPU baselines and their kernel
# stats, attention and GEMM micro-benchmarks, C5-size streamed evaluation.
set -u
export TMPDIR=/tmp
O=gpurun_out/r3b
mkdir -p $O
run() {  # name, seconds, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -1 $O/$name.log | cut -c1-250
  if [ $rc -ne 0 ]; then exit $rc; fi
}
PROF_OUT=$O/prof bash tools/profile.sh || exit 1
run bench_c3 400 python tools/bench_sage.py --steps 20
run bench_c4 400 python tools/bench_sasrec.py --steps 100
run c3_trace 300 rocprofv3 --kernel-trace --stats -d $O/c3 -o run --output-format csv -- python3 tools/bench_sage.py --steps 10 --warmup 3 --cpu-baseline 0
run c4_trace 300 rocprofv3 --kernel-trace --stats -d $O/c4 -o run --output-format csv -- python3 tools/bench_sasrec.py --steps 10 --warmup 3 --cpu-baseline 0
run attn_bench 200 python tools/attn_bench.py --batches 2048 --mixes c4,64
run gemm_bench 200 python tools/gemm_bench.py
run eval_c5 400 python tools/eval_bench.py --users 10000000 --items 1000000 --edges 200000000 --dim 256 --reps 3
