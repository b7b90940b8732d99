#!/bin/bash
# Round-4 A/B libraries of the fused table Adam (furusato_recommend_amd/
# var_adam_*.so, selected with MIREC_LIB; timed by tools/bench_sage.py's
# tg_adam launch time): every object of the current tree except tablegrad.o.
#   var_adam_nt1 / nt2 / nt3   non-temporal loads / stores / both (MIREC_TG_ADAM_NT)
set -e
cd $(dirname $0)/..
make -s -C furusato_recommend_amd/csrc
H="/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Iinclude -Wall -Wno-unused-result --offload-arch=gfx950 -munsafe-fp-atomics"
T=build/var/adam
mkdir -p $T
for k in 1 2 3; do $H -DMIREC_TG_ADAM_NT=$k -c furusato_recommend_amd/csrc/tablegrad.hip -o $T/nt$k.o & done
wait
objs=$(ls build/obj/*.o | grep -v "/tablegrad.o\$")
for k in 1 2 3; do
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs $T/nt$k.o -lpthread -o furusato_recommend_amd/var_adam_nt$k.so
done
ls -la furusato_recommend_amd/var_adam_*.so
