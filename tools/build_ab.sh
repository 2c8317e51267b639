#!/bin/bash
# A/B variants of libzkmi.so: msm.hip rebuilt with extra flags, linked with the
# other in-tree objects into zelana_amd/_ab/libzkmi_<tag>.so (ZKMI_LIB=...).
# usage: tools/build_ab.sh <tag> <hipcc flags...>
set -e
tag=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
B=$ROOT/zelana_amd/build
mkdir -p $ROOT/zelana_amd/_ab /tmp/ab_$tag
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -w "$@" -c $ROOT/zelana_amd/csrc/msm.hip -o /tmp/ab_$tag/msm.o
objs=$(ls $B/*.o | grep -v '/msm.o$')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $ROOT/zelana_amd/_ab/libzkmi_$tag.so /tmp/ab_$tag/msm.o $objs -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo built zelana_amd/_ab/libzkmi_$tag.so
