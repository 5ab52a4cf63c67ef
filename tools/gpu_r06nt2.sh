#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r06nt2; mkdir -p $O
for lib in libgar.so libgar_nt2.so; do
  GAR_LIB_PATH=$R/go-audio-resampler_amd/$lib timeout -k 10 120 python3 tools/bitcmp.py $O/st_$lib.npy 2 20 44100 48000 > /dev/null || exit 1
done
python3 -c "import numpy as np; a=np.load('$O/st_libgar.so.npy'); b=np.load('$O/st_libgar_nt2.so.npy'); print('stereo', a.shape, 'bit-identical' if a.shape==b.shape and np.array_equal(a.view(np.uint32), b.view(np.uint32)) else 'DIFFERENT')"
rm -f $O/*.npy
TAG=r06nt2_ab LIBS="libgar.so libgar_nt2.so" WL=cfg2 SEC=cfg4 ROUNDS=3 bash tools/ab_bench.sh
