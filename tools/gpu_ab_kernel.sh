#!/bin/bash
# A/B of streaming-kernel variants on cfg2 (stereo 600 s), ns256 (256 ch 60 s) and cfg3 (256 ch
# 48k->44.1k VeryHigh 10 s): kernel ms per Process (tools/kbench.py, one child per config, HIP-event
# profile).  VARIANTS is a JSON list fragment of env dicts (GAR_LIB_PATH, knobs); each is run on
# every workload, ROUNDS times interleaved.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-ab}; mkdir -p $O
cd $R
cfgs="[${VARIANTS:-{\}}]"
for r in $(seq ${ROUNDS:-2}); do
  KB_CH=2 KB_SECONDS=600 KB_IN=44100 KB_OUT=48000 KB_Q=3 timeout -k 10 300 python tools/kbench.py "$cfgs" | sed 's/^/cfg2 /' >> $O/ab.txt || exit 1
  KB_CH=256 KB_SECONDS=60 KB_IN=44100 KB_OUT=48000 KB_Q=3 timeout -k 10 300 python tools/kbench.py "$cfgs" | sed 's/^/ns256 /' >> $O/ab.txt || exit 1
  KB_CH=256 KB_SECONDS=10 KB_IN=48000 KB_OUT=44100 KB_Q=4 timeout -k 10 300 python tools/kbench.py "$cfgs" | sed 's/^/cfg3 /' >> $O/ab.txt || exit 1
done
cut -c1-400 $O/ab.txt
exit 0
