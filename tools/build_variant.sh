#!/bin/bash
# Build a libmirec variant with extra -D flags for gemm.hip only:
#   bash tools/build_variant.sh NAME "-DFOO=1 ..."  -> furusato_recommend_amd/NAME.so
set -e
cd $(dirname $0)/..
make -s -C furusato_recommend_amd/csrc
O=build/var_$1
mkdir -p $O
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Iinclude -Wall -Wno-unused-result --offload-arch=gfx950 -munsafe-fp-atomics $2 -c furusato_recommend_amd/csrc/gemm.hip -o $O/gemm.o
objs=$(ls build/obj/*.o | grep -v '/gemm.o$')
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs $O/gemm.o -lpthread -o furusato_recommend_amd/$1.so
