#!/bin/bash
# Kernel sweep on one workload (tools/kbench.py; knob list in the JSON file KB_SWEEP_FILE).
#   KB_CH / KB_SECONDS / KB_IN / KB_OUT / KB_Q select the workload.
mkdir -p gpurun_out
timeout -k 10 600 python tools/kbench.py "$(cat $KB_SWEEP_FILE)" > gpurun_out/${TAG:-attr}.log 2>&1
s=$?; echo "KB_EXIT $s" >> gpurun_out/${TAG:-attr}.log; exit $s
