# Round 5 (p): streamed top-k time split at C2 — product vs a probe with no
# candidate insertion / compaction (the products, staging and test only).
set -u
export TMPDIR=/tmp
E=gpurun_out/r5p
mkdir -p $E
for L in tkA prod; do
  if [ $L = prod ]; then unset MIREC_LIB; else export MIREC_LIB=var/libmirec_$L.so; fi
  timeout -k 10 300 python -u tools/eval_bench.py --reps 10 --dense 0 --check64 0 >> $E/eval.jsonl 2>> $E/eval.log || { echo "eval_bench $L failed"; tail $E/eval.log; exit 1; }
done
unset MIREC_LIB
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-include-regex score_topk --output-format csv -d $E/pmc1 -o run -- python3 tools/eval_bench.py --reps 2 --dense 0 --check64 0 > $E/pmc1.log 2>&1 || { echo "pmc1 rc=$?"; tail -5 $E/pmc1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --kernel-include-regex score_topk --output-format csv -d $E/pmc2 -o run -- python3 tools/eval_bench.py --reps 2 --dense 0 --check64 0 > $E/pmc2.log 2>&1 || { echo "pmc2 rc=$?"; tail -5 $E/pmc2.log; exit 1; }
for p in pmc1 pmc2; do f=$(find $E/$p -name '*counter_collection.csv' | head -1); cp $f $E/${p}.csv; done
rm -rf $E/pmc1 $E/pmc2
cut -c1-200 $E/eval.jsonl
