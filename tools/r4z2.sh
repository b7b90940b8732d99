# Round 4 (session 2n): LightGCN propagation's fused Adam with non-temporal
# W / m / v loads (var_prop_nt.so) against the default build — the C2 line,
# alternating, twice each (no CPU baseline / parity leg).
set -u
E=gpurun_out/r4z2
mkdir -p $E
for rep in 1 2; do
for v in base nt; do
  if [ $v = base ]; then L=""; else L=furusato_recommend_amd/var_prop_nt.so; fi
  MIREC_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline off --parity 0 > $E/c2_$v.$rep.log 2>&1 || { echo "$v rc=$?"; tail -3 $E/c2_$v.$rep.log; exit 1; }
  python3 -c "
import json
d=json.loads([l for l in open('$E/c2_$v.$rep.log') if l.startswith('{')][0])
print('$v', $rep, d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])
" | tee -a $E/summary.txt
done
done
