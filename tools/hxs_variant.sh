#!/bin/bash
# Build libgar_<name>.so with extra flags for the streaming split-f16 kernel objects only (A/B builds):
#   tools/hxs_variant.sh dev "-DGAR_HXS_DEV=1 -DGAR_HXS_QUICK=1"
set -e
name=$1; flags=$2
cd "$(dirname "$0")/../go-audio-resampler_amd"
make -s -j8 >/dev/null
mkdir -p build/$name
CXXFLAGS="-O3 -std=c++17 -fPIC -Wall -Wno-unused-function -fno-slp-vectorize -I../include -Icsrc -I/opt/rocm/include"
units="gar_hxs gar_hxs_i1 gar_hxs_i2 gar_hxt_i1 gar_hxt_i2"
for f in $units; do
  /opt/rocm/bin/hipcc $CXXFLAGS $flags --offload-arch=gfx950 -c csrc/$f.hip -o build/$name/$f.o &
done
wait
objs=$(ls build/*.o | grep -v -E "/gar_hx[st](_i1|_i2)?\.o$")
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o libgar_$name.so $objs build/$name/*.o
echo built libgar_$name.so
