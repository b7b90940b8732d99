# Round 5 (r): attention backward probes at the C4 mix — phase B's dV / dK
# MFMAs replaced by scalar FMAs (atp1), and also its S / dP recompute (atp3):
# how much of the launch the f32 MFMA work sets.  Timing only.
set -u
export TMPDIR=/tmp
E=gpurun_out/r5r
mkdir -p $E
for L in prod atp1 atp3 prod; do
  if [ $L = prod ]; then unset MIREC_LIB; else export MIREC_LIB=var/libmirec_$L.so; fi
  timeout -k 10 120 python tools/attn_bench.py --mixes c4 --batches 2048 --reps 20 > $E/attn_$L.jsonl 2>&1 || { echo "bench $L rc=$?"; tail $E/attn_$L.jsonl; exit 1; }
  echo "$L $(grep packed_bwd $E/attn_$L.jsonl)"
done
