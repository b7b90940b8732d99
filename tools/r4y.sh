# Round 4 (session 2n): fused table Adam with non-temporal loads / stores
# (var_adam_nt1/2/3, tools/build_adam_variants.sh) against the default build:
# the C3 line's tg_adam launch time (HIP events) and step time, twice each.
set -u
E=gpurun_out/r4y
mkdir -p $E
for rep in 1 2; do
for v in base nt1 nt2 nt3; do
  if [ $v = base ]; then L=""; else L=furusato_recommend_amd/var_adam_$v.so; fi
  MIREC_LIB=$L timeout -k 10 200 python tools/bench_sage.py --steps 30 --cpu-baseline 0 > $E/c3_$v.$rep.log 2>&1 || { echo "$v rc=$?"; tail -3 $E/c3_$v.$rep.log; exit 1; }
  python3 -c "
import json
d=json.loads([l for l in open('$E/c3_$v.$rep.log') if l.startswith('{')][0])
print('$v', $rep, d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])
" | tee -a $E/summary.txt
done
done
