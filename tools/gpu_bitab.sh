#!/bin/bash
# Output bits of library variants ($LIBS, the first is the reference) on 256-ch streams (44.1k->48k High,
# 48k->44.1k VeryHigh, 3 / 2 s), then kernel A/B ($WL + $SEC, $ROUNDS rounds).  TAG names the output dir.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/${TAG:-bitab}; mkdir -p $O
for lib in $LIBS; do
  GAR_LIB_PATH=$R/go-audio-resampler_amd/$lib timeout -k 10 120 python3 tools/bitcmp.py $O/up_$lib.npy 256 3 44100 48000 > /dev/null || exit 1
  GAR_LIB_PATH=$R/go-audio-resampler_amd/$lib timeout -k 10 120 python3 tools/bitcmp.py $O/dn_$lib.npy 256 2 48000 44100 > /dev/null || exit 1
done
python3 - $O $LIBS <<'PY' || exit 1
import sys, numpy as np
O, libs = sys.argv[1], sys.argv[2:]
bad = 0
for k in ("up", "dn"):
    a = np.load(f"{O}/{k}_{libs[0]}.npy")
    for v in libs[1:]:
        b = np.load(f"{O}/{k}_{v}.npy")
        same = a.shape == b.shape and np.array_equal(a.view(np.uint32), b.view(np.uint32))
        bad += not same
        print(k, v, a.shape, "bit-identical" if same else "DIFFERENT max %g" % float(np.abs(a - b).max()))
sys.exit(1 if bad else 0)
PY
s=$?; rm -f $O/*.npy; [ $s -eq 0 ] || exit $s
TAG=${TAG:-bitab}_ab LIBS="$LIBS" WL=${WL:-ns256} SEC=${SEC:-cfg2,cfg3,cfg4} ROUNDS=${ROUNDS:-2} bash tools/ab_bench.sh || exit 1
