#!/bin/bash
# Round-4 A/B libraries of the sorted table-gradient sum (furusato_recommend_amd/
# var_tg_*.so, selected with MIREC_LIB; timed by tools/tg_bench.py): every
# object of the current tree except tablegrad.o.
#   var_tg_head   tablegrad.hip as of the last commit
#   var_tg_ch4 / var_tg_ch16   the current source with 4 / 16 entries per chunk
#   var_tg_sort11 the current source sorting 11 bits per onesweep pass (two passes at C3)
set -e
cd $(dirname $0)/..
make -s -C furusato_recommend_amd/csrc
H="/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Iinclude -Wall -Wno-unused-result --offload-arch=gfx950 -munsafe-fp-atomics"
T=build/var/tg
mkdir -p $T
git show HEAD:furusato_recommend_amd/csrc/tablegrad.hip > $T/tablegrad_head.hip
cp furusato_recommend_amd/csrc/common.h $T/
$H -c $T/tablegrad_head.hip -o $T/head.o &
$H -DMIREC_TG_CHUNK=4 -c furusato_recommend_amd/csrc/tablegrad.hip -o $T/ch4.o &
$H -DMIREC_TG_CHUNK=16 -c furusato_recommend_amd/csrc/tablegrad.hip -o $T/ch16.o &
$H -DMIREC_TG_SORT_BITS=11 -c furusato_recommend_amd/csrc/tablegrad.hip -o $T/sort11.o &
wait
link() {  # name, variant object
  objs=$(ls build/obj/*.o | grep -v "/tablegrad.o\$")
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs $2 -lpthread -o furusato_recommend_amd/$1.so
}
link var_tg_head $T/head.o
link var_tg_ch4 $T/ch4.o
link var_tg_ch16 $T/ch16.o
link var_tg_sort11 $T/sort11.o
ls -la furusato_recommend_amd/var_tg_*.so
