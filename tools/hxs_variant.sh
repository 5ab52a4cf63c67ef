#!/bin/bash
# Build libgar_<name>.so with extra flags for some objects only (A/B builds; default the streaming
# split-f16 kernel units, UNITS overrides):
#   tools/hxs_variant.sh dev "-DGAR_HXS_DEV=1 -DGAR_HXS_QUICK=1"
#   UNITS="gar_kernels gar_bg_f64" tools/hxs_variant.sh bgdev "-DGAR_BG_DEV=1"
set -e
name=$1; flags=$2
cd "$(dirname "$0")/../go-audio-resampler_amd"
[ -n "$SKIPMAKE" ] || make -s -j8 >/dev/null
mkdir -p build/$name
CXXFLAGS="-O3 -std=c++17 -fPIC -Wall -Wno-unused-function -fno-slp-vectorize -I../include -Icsrc -I/opt/rocm/include"
units=${UNITS:-"gar_hxs gar_hxs_i1 gar_hxs_i2 gar_hxt_i1 gar_hxt_i2"}
for f in $units; do
  /opt/rocm/bin/hipcc $CXXFLAGS $flags --offload-arch=gfx950 -c csrc/$f.hip -o build/$name/$f.o &
done
wait
objs=$(for o in build/*.o; do b=$(basename $o .o); case " $units " in *" $b "*) ;; *) echo $o;; esac; done)
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o libgar_$name.so $objs build/$name/*.o
echo built libgar_$name.so
