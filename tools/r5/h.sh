# Round 5 (h): table-gradient pass 1 A/B — HEAD (row gathers as flat loads),
# tgg (global loads), product (global loads + the extension batch as
# LDS-DMA beside the chunk's own rows); table-gradient tests first, then
# tg_bench twice per build, then one rocprofv3 kernel-stats pass per build.
set -u
export TMPDIR=/tmp
E=gpurun_out/r5h
mkdir -p $E
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 500 --timeout-method thread -k "table_grad or tablegrad or sage" > $E/pytest_tg.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 $E/pytest_tg.log
[ $rc = 0 ] || exit $rc
for rep in 1 2; do
  for L in tgb tgg prod; do
    if [ $L = prod ]; then unset MIREC_LIB; else export MIREC_LIB=var/libmirec_$L.so; fi
    timeout -k 10 200 python tools/tg_bench.py --reps 50 > $E/tg_$L.json 2>> $E/tg_ab.log || { echo "tg_bench $L failed"; tail $E/tg_ab.log; exit 1; }
    echo "$L $(cat $E/tg_$L.json)" | tee -a $E/tg_ab.jsonl
  done
done
for L in tgb tgg prod; do
  if [ $L = prod ]; then unset MIREC_LIB; else export MIREC_LIB=var/libmirec_$L.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $E/prof_$L -o run -- python3 tools/tg_bench.py --reps 20 > $E/prof_$L.log 2>&1 || { echo "prof $L failed"; tail $E/prof_$L.log; exit 1; }
done
for L in tgb tgg prod; do echo "== $L"; find $E/prof_$L -name '*kernel_stats.csv' -exec grep -h "tg_sum\|tg_adam\|tg_fixup\|Onesweep\|tg_plan" {} \; | cut -c1-160; done
