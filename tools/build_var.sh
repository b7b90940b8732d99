#!/bin/bash
# A/B build: the current csrc/ tree linked into var/libmirec_<name>.so (the
# objects of build/obj, with the named sources recompiled from csrc/ as they
# are now), so tools/*_bench.py can time it with MIREC_LIB beside the
# product library.  Usage: bash tools/build_var.sh <name> <file.hip> ...
set -eu
name=$1; shift
H="/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -I$PWD/include -Wall -Wno-unused-result --offload-arch=gfx950 -munsafe-fp-atomics"
T=build/var_$name
rm -rf $T && mkdir -p $T var
cp build/obj/*.o $T/
for f in "$@"; do
  $H -c furusato_recommend_amd/csrc/$f -o $T/${f%.hip}.o
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $T/*.o -lpthread -o var/libmirec_$name.so
echo var/libmirec_$name.so
