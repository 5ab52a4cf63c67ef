#!/bin/bash
# r06w: transposed output tiles (libgar_tr) and + mixed split (libgar_trmix) vs libgar.so: output bits
# of 256-ch streams (44.1k->48k High, 48k->44.1k VeryHigh), then kernel A/B
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r06w; mkdir -p $O
for lib in libgar.so libgar_tr.so libgar_trmix.so; do
  GAR_LIB_PATH=$R/go-audio-resampler_amd/$lib timeout -k 10 120 python3 tools/bitcmp.py $O/up_$lib.npy 256 3 44100 48000 || exit 1
  GAR_LIB_PATH=$R/go-audio-resampler_amd/$lib timeout -k 10 120 python3 tools/bitcmp.py $O/dn_$lib.npy 256 2 48000 44100 || exit 1
done
python3 - <<'PY' || exit 1
import numpy as np
O = "gpurun_out/r06w"
for k in ("up", "dn"):
    a = np.load(f"{O}/{k}_libgar.so.npy")
    for v in ("libgar_tr.so", "libgar_trmix.so"):
        b = np.load(f"{O}/{k}_{v}.npy")
        same = a.shape == b.shape and np.array_equal(a.view(np.uint32), b.view(np.uint32))
        print(k, v, a.shape, "bit-identical" if same else "DIFFERENT", "" if same else float(np.abs(a - b).max()))
PY
rm -f $O/*.npy
TAG=r06w_ab LIBS="libgar.so libgar_tr.so libgar_trmix.so" WL=ns256 SEC=cfg2,cfg3 ROUNDS=2 bash tools/ab_bench.sh || exit 1
