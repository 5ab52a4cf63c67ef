#!/bin/bash
# hxq_kernel phase stamps (development library): stereo and 256-channel 4096-frame streams.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04g; mkdir -p $O; L=$O/prof.txt
D=$R/go-audio-resampler_amd/libgar_dev.so
run() { echo "== $*" >> $L; env "$@" >> $L 2>&1; }
run GAR_LIB_PATH=$D GAR_HXS_PROF=1 P_N=300 timeout -k 10 90 python tools/stream_probe.py || exit 1
run GAR_LIB_PATH=$D GAR_HXS_PROF=1 GAR_HXQ_NR=2 P_N=300 timeout -k 10 90 python tools/stream_probe.py || exit 1
run GAR_LIB_PATH=$D GAR_HXS_PROF=1 P_CH=256 P_N=100 timeout -k 10 90 python tools/stream_probe.py || exit 1
cat $L
