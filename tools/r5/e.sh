# Round 5 (e): timing probes of the streamed top-k (outputs discarded):
# without the candidate filter, with 1/8 of the MFMAs, without the
# mid-tile barrier.
set -u
export TMPDIR=/tmp
E=gpurun_out/r5e
mkdir -p $E
for L in tkold prod tknoflt tknocmp; do
  if [ $L = prod ]; then unset MIREC_LIB; else export MIREC_LIB=var/libmirec_$L.so; fi
  timeout -k 10 300 python -u tools/eval_bench.py --reps 10 --dense 0 --check64 0 >> $E/probe.jsonl 2>> $E/probe.log || { echo "eval_bench $L failed"; tail $E/probe.log; exit 1; }
done
cat $E/probe.jsonl | cut -c1-200
