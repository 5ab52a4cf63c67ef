#!/bin/bash
# Build libgar_<name>.so with extra flags for the hxs kernel objects only (A/B builds):
#   tools/hxs_variant.sh l4d2 "-DGAR_HXS_L=4 -DGAR_HXS_D=2"
set -e
name=$1; flags=$2
cd "$(dirname "$0")/../go-audio-resampler_amd"
make -s -j8 >/dev/null
mkdir -p build/$name
CXXFLAGS="-O3 -std=c++17 -fPIC -Wall -Wno-unused-function -fno-slp-vectorize -I../include -Icsrc -I/opt/rocm/include"
for f in gar_hxs gar_hxs_i1 gar_hxs_i2; do
  /opt/rocm/bin/hipcc $CXXFLAGS $flags --offload-arch=gfx950 -c csrc/$f.hip -o build/$name/$f.o &
done
wait
objs=$(ls build/*.o | grep -v -E "/gar_hxs(_i1|_i2)?\.o$")
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o libgar_$name.so $objs build/$name/*.o
echo built libgar_$name.so
