#!/bin/bash
# A/B builds of libvbc: recompile one translation unit with extra defines and link it with the other
# objects of the in-tree build.  Usage: tools/exp/build_variant.sh NAME TU "-DFOO=1 -DBAR=2"
# -> tools/exp/libs/libvbc_NAME.so (tools/ab.py "@lib=tools/exp/libs/libvbc_NAME.so").
set -e
name=$1; tu=$2; defs=$3
cd "$(dirname "$0")/../../sparsematrixvbcs.jl_amd"
mkdir -p ../tools/exp/libs /tmp/vbc_variant_$name
objs=""
for o in build/*.o; do
  [ "$(basename $o .o)" = "$tu" ] && continue
  objs="$objs $o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fvisibility=hidden -Wall -Wno-unused-result \
  -I../include -Icsrc $defs -c csrc/$tu.hip -o /tmp/vbc_variant_$name/$tu.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared $objs /tmp/vbc_variant_$name/$tu.o -o ../tools/exp/libs/libvbc_$name.so \
  -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo built tools/exp/libs/libvbc_$name.so
