# Round 5 (d): instruction counters of the streamed top-k kernel (C2 batch),
# round-4 build and product build.
set -u
export TMPDIR=/tmp
E=gpurun_out/r5d
mkdir -p $E
for L in tkold prod; do
  if [ $L = prod ]; then unset MIREC_LIB; else export MIREC_LIB=var/libmirec_$L.so; fi
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_MFMA SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM --kernel-include-regex score_topk -d $E/i_$L -o run --output-format csv -- python3 tools/eval_bench.py --reps 1 --dense 0 --check64 0 > $E/i_$L.log 2>&1 || { echo "$L rc=$?"; tail $E/i_$L.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVES --kernel-include-regex score_topk -d $E/c_$L -o run --output-format csv -- python3 tools/eval_bench.py --reps 1 --dense 0 --check64 0 > $E/c_$L.log 2>&1 || { echo "$L rc=$?"; tail $E/c_$L.log; exit 1; }
done
echo done
