#!/bin/bash
# Measurement evidence on one GPU box, as named legs:
#
#   bash tools/evidence.sh [leg ...]        (default: tests c2 prof c3 c4 c3prof c4prof)
#
# Output under gpurun_out/${EV:-ev}/.  Every GPU step runs under its own time
# limit and a failing step ends the script (nothing more touches the GPU).
# rocprofv3 writes CSV; per-dispatch trace CSVs are deleted so only the
# *_stats.csv (and counter CSVs of the PMC passes) stay.  The summaries that
# profiles/ keeps come from these directories (profiles/README.md).
#
#   tests      the whole GPU suite in one process               -> pytest.log
#   mark=EXPR  the GPU tests selected by -k EXPR ('+' for spaces: mark=a+or+b), verbose -> pytest_k.log
#   smoke      __graft_entry__.smoke()                           -> smoke.log
#   c2         the headline bench line (bench.py defaults: roofline, CPU
#              baseline, oracle parity leg, Recall@20)           -> bench_c2.log
#   c2quick    the C2 line without the CPU baseline and Recall legs (oracle parity kept)
#   prof       C2 rocprofv3 passes: kernel stats, FETCH_SIZE, WRITE_SIZE of
#              prop_kernel (tools/profile.sh), summarised        -> prof/, summary.json
#   c2prof     kernel stats of 13 C2 steps (no CPU / parity / Recall legs)
#   c3 / c4    GraphSAGE C3 / SASRec C4 lines with CPU baselines -> bench_c3.log, bench_c4.log
#   c3prof / c4prof   kernel stats of the C3 step / the captured C4 step
#   zipf       the C2 Zipf-popularity graph: line + kernel stats
#   c4nodes    the captured C4 step's HIP graph by node kind (memcpy / memset /
#              kernels; tools/c4_graph_nodes.py)                -> c4_graph_nodes.log
#   rehearse2 / rehearse8   bench.py --gpus N --rehearse (N ranks on one GPU,
#              gloo): the DP parity and Recall@20 legs   -> bench_c2_rehearse_dpN.log
#   c5         LightGCN-3 d=256 10 M x 1 M / 200 M on one GPU   -> bench_c5.log
#   pmc_tg     FETCH / WRITE of the C3 table-gradient sum vs its algorithmic
#              bytes (tools/tg_sum_bytes.py)                     -> pmc_tg_sum.json
#   world_c3   the C3 world simulation (W = 1 over 30 steps, W = 8 with 2 / 3
#              micro-batches and the plain fetch exchange)
#   trace_c3   device timeline of one simulated pipelined C3 step (W = 8, C = 2):
#              rocprofv3 --kernel-trace + tools/trace_step.py  -> trace_c3_step.txt
#   world_c2   rank 0's C2 step at W = 1..8 (sparse / sharded)
#   world_c5   rank 0's C5 step (10 M x 1 M / 200 M, d = 256) at W = 1..8 (sparse / sharded)
#   eval       streamed evaluation at C2 with the float64 near-tie check
#   eval_d256  the streamed evaluation at d = 256 (2 M x 1 M, the D > 128 path)
#   attn       attention kernels at the C4 length mix
#   attn_pmc   SQ counters of the packed attention backward (two passes)
#   topk_pmc   SQ counters of the streamed top-k at C2 (two passes)
#   gemm_pmc   SQ counters of the resident-B GEMM (gemm_bench shapes, two passes)
#   tg         the C3 table-gradient accumulate alone (tools/tg_bench.py)
#   gemm       the GEMM shapes of C3 / C4 and 4096^3
set -u
export TMPDIR=/tmp
E=gpurun_out/${EV:-ev}
mkdir -p $E
LEGS=${*:-tests c2 prof c3 c4 c3prof c4prof}

run() {  # run LIMIT LOG CMD...: one GPU step, its own limit, stop on failure
  local lim=$1 log=$2
  shift 2
  timeout -k 10 "$lim" "$@" > "$log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then
    echo "FAILED rc=$rc: $*"
    tail -20 "$log"
    exit $rc
  fi
}

lines() { grep '^{' "$1" | cut -c1-${2:-400} || true; }

for leg in $LEGS; do
  echo "== $leg"
  case $leg in
    tests)
      run 1100 $E/pytest.log python -u -m pytest tests -m gpu -q -rf --timeout 500 --timeout-method thread
      tail -3 $E/pytest.log ;;
    mark=*)
      run 900 $E/pytest_k.log python -u -m pytest tests -m gpu -x -v -s --timeout 500 --timeout-method thread -k "$(echo "${leg#mark=}" | tr '+' ' ')"
      tail -5 $E/pytest_k.log ;;
    smoke)
      run 300 $E/smoke.log python -c "import __graft_entry__ as g; g.smoke()"
      tail -3 $E/smoke.log ;;
    c2)
      run 700 $E/bench_c2.log python bench.py
      lines $E/bench_c2.log 600 ;;
    c2quick)
      run 400 $E/bench_c2_quick.log python bench.py --cpu-baseline off --quality-steps 0
      lines $E/bench_c2_quick.log 600 ;;
    prof)
      PROF_OUT=$E/prof bash tools/profile.sh || exit 1
      find $E/prof -name "*kernel_trace.csv" -delete
      python tools/summarize_prof.py $E/prof ${TAG:-ev} > $E/summary.log 2>&1 || { echo "summarize failed"; tail $E/summary.log; } ;;
    c3)
      run 400 $E/bench_c3.log python tools/bench_sage.py --steps 20
      lines $E/bench_c3.log ;;
    c4)
      run 400 $E/bench_c4.log python tools/bench_sasrec.py --steps 100
      lines $E/bench_c4.log ;;
    c2prof)
      run 300 $E/c2prof.log rocprofv3 --kernel-trace --stats -d $E/c2 -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --cpu-baseline off --quality-steps 0 --parity 0
      find $E/c2 -name "*kernel_trace.csv" -delete ;;
    c3prof)
      run 300 $E/c3prof.log rocprofv3 --kernel-trace --stats -d $E/c3 -o run --output-format csv -- python3 tools/bench_sage.py --steps 10 --warmup 3 --cpu-baseline 0
      find $E/c3 -name "*kernel_trace.csv" -delete ;;
    c4prof)
      run 300 $E/c4prof.log rocprofv3 --kernel-trace --stats -d $E/c4 -o run --output-format csv -- python3 tools/bench_sasrec.py --steps 10 --warmup 3 --cpu-baseline 0
      find $E/c4 -name "*kernel_trace.csv" -delete ;;
    zipf)
      run 300 $E/bench_c2_zipf.log python bench.py --kind zipf --steps 20 --warmup 3 --cpu-baseline off --quality-steps 0 --parity 0
      lines $E/bench_c2_zipf.log
      run 300 $E/zipf.log rocprofv3 --kernel-trace --stats -d $E/zipf -o run --output-format csv -- python3 bench.py --kind zipf --steps 10 --warmup 3 --cpu-baseline off --quality-steps 0 --parity 0
      find $E/zipf -name "*kernel_trace.csv" -delete ;;
    c4nodes)
      run 300 $E/c4_graph_nodes.log python tools/c4_graph_nodes.py --out $E/c4_graph.dot
      lines $E/c4_graph_nodes.log 3000 ;;
    rehearse2|rehearse8)
      # the N-rank bench on one GPU (gloo): parity leg (bitwise replicas +
      # union-batch replay on rank 0) and the DataParallel Recall@20 leg
      N=${leg#rehearse}
      Q=$([ "$N" = 8 ] && echo 1000 || echo 3000)
      run 700 $E/bench_c2_rehearse_dp$N.log python bench.py --gpus $N --rehearse --steps 5 --warmup 2 --quality-steps $Q
      lines $E/bench_c2_rehearse_dp$N.log 600 ;;
    c5)
      run 900 $E/bench_c5.log python bench.py --users 10000000 --items 1000000 --edges 200000000 --dim 256 --steps 5 --warmup 2 --cpu-baseline off --quality-steps 0 --parity 0
      lines $E/bench_c5.log ;;
    pmc_tg)
      timeout -k 10 200 python -u tools/tg_sum_bytes.py > $E/tg_counts.json 2> $E/tg_counts.log || { echo "tg counts rc=$?"; exit 1; }
      timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex tg_sum -d $E/tgf -o run --output-format csv -- python3 tools/bench_sage.py --steps 5 --warmup 2 --cpu-baseline 0 > $E/tgf.log 2>&1 || { echo "pmc fetch rc=$?"; exit 1; }
      timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex tg_sum -d $E/tgw -o run --output-format csv -- python3 tools/bench_sage.py --steps 5 --warmup 2 --cpu-baseline 0 > $E/tgw.log 2>&1 || { echo "pmc write rc=$?"; exit 1; }
      python tools/tg_sum_bytes.py --counts $E/tg_counts.json --fetch $E/tgf --write $E/tgw --out $E/pmc_tg_sum.json
      find $E/tgf $E/tgw -name "*kernel_trace.csv" -delete ;;
    world_c3)
      timeout -k 10 900 python -u tools/bench_world_sim.py --model sage --worlds 1,8 --exchanges fetch --microbatches 2,3 --steps 30 > $E/world_sim_c3.jsonl 2> $E/world_sim_c3.log || { echo "world sim rc=$?"; tail $E/world_sim_c3.log; exit 1; }
      lines $E/world_sim_c3.jsonl 300 ;;
    trace_c3)
      run 300 $E/trace_c3.log rocprofv3 --kernel-trace --output-format csv -d $E/trc3 -o run -- python3 tools/bench_world_sim.py --model sage --worlds 8 --exchanges fetch --microbatches 2 --steps 3 --warmup 2
      f=$(find $E/trc3 -name '*kernel_trace.csv' | head -1)
      # the pipelined run's steps come first (7 + 5 bpr_sample markers); step 11 is its last
      python3 tools/trace_step.py "$f" --nth 11 --width 90 > $E/trace_c3_step.txt
      rm -rf $E/trc3
      tail -1 $E/trace_c3_step.txt ;;
    world_c2)
      timeout -k 10 900 python -u tools/bench_world_sim.py --modes sparse,sharded > $E/world_sim_c2.jsonl 2> $E/world_sim_c2.log || { echo "world sim rc=$?"; tail $E/world_sim_c2.log; exit 1; }
      lines $E/world_sim_c2.jsonl 300 ;;
    world_c5)
      timeout -k 10 1000 python -u tools/bench_world_sim.py --users 10000000 --items 1000000 --edges 200000000 --dim 256 --modes sparse,sharded --steps 5 --warmup 2 > $E/world_sim_c5.jsonl 2> $E/world_sim_c5.log || { echo "world sim rc=$?"; tail $E/world_sim_c5.log; exit 1; }
      lines $E/world_sim_c5.jsonl 300 ;;
    eval)
      run 600 $E/eval_c2.log python -u tools/eval_bench.py --reps 10
      lines $E/eval_c2.log 300 ;;
    eval_d256)
      run 600 $E/eval_d256.log python -u tools/eval_bench.py --users 2000000 --items 1000000 --edges 40000000 --dim 256 --batch 2000 --reps 3 --dense 0
      lines $E/eval_d256.log 300 ;;
    attn)
      run 400 $E/attn.log python -u tools/attn_bench.py --mixes c4 --batches 2048
      lines $E/attn.log 300 ;;
    attn_pmc|topk_pmc|gemm_pmc)
      if [ $leg = attn_pmc ]; then K=attn_bwd_packed; CMD="python3 tools/attn_bench.py --mixes c4 --batches 2048 --reps 3"
      elif [ $leg = gemm_pmc ]; then K=gemm_nt_res; CMD="python3 tools/gemm_bench.py --reps 3"
      else K=score_topk; CMD="python3 tools/eval_bench.py --reps 2 --dense 0 --check64 0"; fi
      P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
      P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
      n=0
      for P in "$P1" "$P2"; do
        n=$((n + 1))
        timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex $K --output-format csv -d $E/${leg}$n -o run -- $CMD > $E/${leg}$n.log 2>&1 || { echo "$leg pass $n rc=$?"; tail -5 $E/${leg}$n.log; exit 1; }
        cp $(find $E/${leg}$n -name '*counter_collection.csv' | head -1) $E/${leg}$n.csv
        rm -rf $E/${leg}$n
      done ;;
    tg)
      run 200 $E/tg.json python tools/tg_bench.py --reps 50
      cat $E/tg.json ;;
    gemm)
      run 400 $E/gemm.log python -u tools/gemm_bench.py
      lines $E/gemm.log 300 ;;
    *)
      echo "unknown leg $leg"; exit 2 ;;
  esac
done
du -sh $E
echo "evidence ok: $LEGS"
