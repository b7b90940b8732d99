# Same-box A/B of gemm_tn row-slice sizes in the C4 step: build the variant with
# hipcc -DMIREC_TN_MINROWS=256 (gemm.hip) into furusato_recommend_amd/libmirec_tn256.so.
set -e
O=gpurun_out/tn
mkdir -p $O
for lib in libmirec.so libmirec_tn256.so libmirec.so libmirec_tn256.so; do
  echo "lib=$lib" >> $O/gemm.txt
  MIREC_LIB=$PWD/furusato_recommend_amd/$lib timeout -k 10 120 python tools/gemm_bench.py 2>/dev/null | grep -E "_dw" | cut -c1-120 >> $O/gemm.txt
  MIREC_LIB=$PWD/furusato_recommend_amd/$lib timeout -k 10 200 python tools/bench_sasrec.py --steps 50 --warmup 5 --cpu-baseline 0 2>/dev/null | grep '^{' | cut -c1-170 >> $O/gemm.txt
done
echo ok
