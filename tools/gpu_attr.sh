#!/bin/bash
# Attribution sweep of the streaming kernel on one workload (dev build: GAR_HXS_DEV=1).
#   KB_CH / KB_SECONDS / KB_IN / KB_OUT / KB_Q select the workload; KB_SWEEP the knob list.
mkdir -p gpurun_out
timeout -k 10 600 python tools/kbench.py "$KB_SWEEP" > gpurun_out/${TAG:-attr}.log 2>&1
s=$?; echo "KB_EXIT $s" >> gpurun_out/${TAG:-attr}.log; exit $s
