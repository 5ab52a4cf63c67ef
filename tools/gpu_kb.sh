#!/bin/bash
# kernel-knob sweep on the bench workload: tools/kbench.py '<json list of env dicts>'
mkdir -p gpurun_out
timeout -k 10 900 python tools/kbench.py "$KB_SWEEP" > gpurun_out/kbench.log 2>&1
s=$?; echo "KB_EXIT $s" >> gpurun_out/kbench.log; exit $s
