#!/bin/bash
# A/B build: var/libmirec_<name>.so = the objects of build/obj (the product
# build) with the named sources recompiled — from csrc/ as they are now, or
# from another file given as <src>=<path> (e.g. a `git show` of an older
# revision) — so tools/*_bench.py can time it with MIREC_LIB beside the
# product library.  Usage: bash tools/build_var.sh <name> <file.hip>[=<path>] ...
set -eu
name=$1; shift
C=furusato_recommend_amd/csrc
H="/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -I$PWD/include -I$PWD/$C -Wall -Wno-unused-result --offload-arch=gfx950 -munsafe-fp-atomics"
make -C $C -s
T=build/var_$name
rm -rf $T && mkdir -p $T var
cp build/obj/*.o $T/
for spec in "$@"; do
  f=${spec%%=*}
  src=$C/$f
  [ "$spec" != "$f" ] && src=${spec#*=}
  $H -x hip -c $src -o $T/${f%.hip}.o
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $T/*.o -lpthread -o var/libmirec_$name.so
echo var/libmirec_$name.so
