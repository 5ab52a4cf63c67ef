#!/bin/bash
# r06z: the 32-channel-block build (FMT 5, default) -- output bits against GAR_HXT_WIDE=0 (16-channel
# blocks) in the same library, the whole -m gpu suite and smoke, then the driver's bench command.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r06z; mkdir -p $O
for w in 0 1; do
  GAR_HXT_WIDE=$w timeout -k 10 120 python3 tools/bitcmp.py $O/up_$w.npy 256 3 44100 48000 > /dev/null || exit 1
  GAR_HXT_WIDE=$w timeout -k 10 120 python3 tools/bitcmp.py $O/dn_$w.npy 256 2 48000 44100 > /dev/null || exit 1
  GAR_HXT_WIDE=$w timeout -k 10 120 python3 tools/bitcmp.py $O/w64_$w.npy 64 2 44100 96000 > /dev/null || exit 1
done
python3 - <<'PY' | tee $O/bits.txt || exit 1
import numpy as np, sys
bad = 0
for k in ("up", "dn", "w64"):
    a, b = np.load(f"gpurun_out/r06z/{k}_0.npy"), np.load(f"gpurun_out/r06z/{k}_1.npy")
    same = a.shape == b.shape and np.array_equal(a.view(np.uint32), b.view(np.uint32))
    bad += not same
    print(k, a.shape, "bit-identical (GAR_HXT_WIDE 0 vs 1)" if same else "DIFFERENT")
sys.exit(1 if bad else 0)
PY
rm -f $O/*.npy
TAG=r06z BENCH=${BENCH:-1} PROF=${PROF:-0} PMC=${PMC:-0} bash tools/gpu_run.sh
