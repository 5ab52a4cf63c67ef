#!/bin/bash
# hxq variants (GAR_HXQ_OPT: 1 barrier after the first batch, 2 buffer-load history keep) in one run:
# dev-library phase stamps and C-ABI device-call times, alternating to cancel drift.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r04j}; mkdir -p $O
P=$O/prof.txt; C=$O/cabi.txt
D=$R/go-audio-resampler_amd/libgar_dev.so
for rep in 1 2; do
for v in 0 1 2 3; do
  echo "== rep $rep GAR_HXQ_OPT=$v" >> $P
  GAR_HXQ_OPT=$v GAR_LIB_PATH=$D GAR_HXS_PROF=1 P_N=300 timeout -k 10 90 python tools/stream_probe.py >> $P 2>&1 || exit 1
  echo "== rep $rep GAR_HXQ_OPT=$v" >> $C
  GAR_HXQ_OPT=$v timeout -k 10 120 ./tools/cabi_stream 4096 30 2 >> $C 2>&1 || exit 1
done
done
grep -v amdgpu.ids $P | grep -v "loader\|^hxs prof\|slowest"
grep "==\|\"device\"\|host_multi" $C
