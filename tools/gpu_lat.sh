#!/bin/bash
# Small-launch latency probes: streaming calls and cfg5 chunks, kernarg placement, dev phase stamps.
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O; L=$O/lat.log; : > $L
D=$GRAFT_REPO_ROOT/go-audio-resampler_amd/libgar_dev.so
run() { echo "== $*" >> $L; env "$@" >> $L 2>&1; }
run P_N=600 timeout -k 10 60 python tools/stream_probe.py || exit 1
run HIP_FORCE_DEV_KERNARG=1 P_N=600 timeout -k 10 60 python tools/stream_probe.py || exit 1
run HIP_FORCE_DEV_KERNARG=0 P_N=600 timeout -k 10 60 python tools/stream_probe.py || exit 1
run P_N=300 timeout -k 10 60 python tools/cfg5_probe.py || exit 1
run HIP_FORCE_DEV_KERNARG=1 P_N=300 timeout -k 10 60 python tools/cfg5_probe.py || exit 1
run GAR_LIB_PATH=$D GAR_HXS_PROF=1 P_N=600 timeout -k 10 60 python tools/stream_probe.py || exit 1
run GAR_LIB_PATH=$D GAR_HXS_PROF=1 KB_SECONDS=600 KB_CH=2 timeout -k 10 60 python tools/kone.py || exit 1
exit 0
