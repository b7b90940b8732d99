# Same-box A/B of library builds (MIREC_LIB) on the C3 and C4 steps:
#   bash tools/ab_libs.sh "c3libs..." "c4libs..."   (names under furusato_recommend_amd/)
set -e
O=gpurun_out/ab
mkdir -p $O
for lib in $1; do
  MIREC_LIB=$PWD/furusato_recommend_amd/$lib timeout -k 10 200 python tools/bench_sage.py --steps 30 --warmup 5 --cpu-baseline 0 2>/dev/null | grep '^{' | cut -c1-150 | sed "s/^/$lib /" >> $O/c3.txt
done
for lib in $2; do
  MIREC_LIB=$PWD/furusato_recommend_amd/$lib timeout -k 10 200 python tools/bench_sasrec.py --steps 50 --warmup 5 --cpu-baseline 0 2>/dev/null | grep '^{' | cut -c1-150 | sed "s/^/$lib /" >> $O/c4.txt
done
echo ok
