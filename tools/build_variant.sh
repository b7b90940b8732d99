#!/bin/bash
# Build a libmirec variant with extra -D flags for one source (default gemm):
#   bash tools/build_variant.sh NAME "-DFOO=1 ..." [gemm|attention|...]
#   -> furusato_recommend_amd/NAME.so  (MIREC_LIB=... selects it)
set -e
cd $(dirname $0)/..
make -s -C furusato_recommend_amd/csrc
SRC=${3:-gemm}
O=build/var_$1
mkdir -p $O
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Iinclude -Wall -Wno-unused-result --offload-arch=gfx950 -munsafe-fp-atomics $2 -c furusato_recommend_amd/csrc/$SRC.hip -o $O/$SRC.o
objs=$(ls build/obj/*.o | grep -v "/$SRC.o\$")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs $O/$SRC.o -lpthread -o furusato_recommend_amd/$1.so
