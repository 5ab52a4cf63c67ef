#!/bin/bash
# C-ABI streaming numbers without Python (tools/cabi_stream.cpp): stereo and 256-channel 4096-frame
# calls through the device API and the host ProcessMulti path, plus the reference's ProcessInto shape.
TAG=${TAG:-r03}
O="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$O"
timeout -k 10 240 ./tools/cabi_stream 4096 60 2 > "$O/${TAG}_cabi_stereo.txt" 2>&1
s=$?; echo "EXIT $s" >> "$O/${TAG}_cabi_stereo.txt"; [ $s -eq 0 ] || exit $s
timeout -k 10 240 ./tools/cabi_stream 4096 10 256 > "$O/${TAG}_cabi_256.txt" 2>&1
s=$?; echo "EXIT $s" >> "$O/${TAG}_cabi_256.txt"; exit $s
