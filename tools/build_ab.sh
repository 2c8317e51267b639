#!/bin/bash
# A/B variants of libzkmi.so: one translation unit rebuilt with extra flags,
# linked with the other in-tree objects into zelana_amd/_ab/libzkmi_<tag>.so
# (load it with ZKMI_LIB=...).
# usage: [SRC=ntt] tools/build_ab.sh <tag> <hipcc flags...>     (SRC default: msm)
set -e
tag=$1; shift
SRC=${SRC:-msm}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
B=$ROOT/zelana_amd/build
mkdir -p $ROOT/zelana_amd/_ab /tmp/ab_$tag
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -w "$@" -c $ROOT/zelana_amd/csrc/$SRC.hip -o /tmp/ab_$tag/$SRC.o
objs=$(ls $B/*.o | grep -v "/$SRC.o\$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $ROOT/zelana_amd/_ab/libzkmi_$tag.so /tmp/ab_$tag/$SRC.o $objs -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo built zelana_amd/_ab/libzkmi_$tag.so
