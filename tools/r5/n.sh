# Round 5 (n): SQ counters of the attention backward at the C4 mix.
set -u
export TMPDIR=/tmp
E=gpurun_out/r5n
mkdir -p $E
timeout -k 10 120 python tools/attn_bench.py --mixes c4 --batches 2048 --reps 20 > $E/attn.jsonl 2>&1 || { echo "bench rc=$?"; tail $E/attn.jsonl; exit 1; }
grep packed_bwd $E/attn.jsonl
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-include-regex attn_bwd_packed --output-format csv -d $E/pmc1 -o run -- python3 tools/attn_bench.py --mixes c4 --batches 2048 --reps 3 > $E/pmc1.log 2>&1 || { echo "pmc1 rc=$?"; tail -5 $E/pmc1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --kernel-include-regex attn_bwd_packed --output-format csv -d $E/pmc2 -o run -- python3 tools/attn_bench.py --mixes c4 --batches 2048 --reps 3 > $E/pmc2.log 2>&1 || { echo "pmc2 rc=$?"; tail -5 $E/pmc2.log; exit 1; }
for p in pmc1 pmc2; do f=$(find $E/$p -name '*counter_collection.csv' | head -1); cp $f $E/${p}.csv; done
rm -rf $E/pmc1 $E/pmc2
