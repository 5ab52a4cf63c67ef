#!/bin/bash
# GPU tests; cfg5 probe (bg_rt 8-load batches); hxq waves-per-workgroup A/B (C-ABI numbers + dev stamps).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r04i}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  ${TESTS:-tests/test_gpu_layouts.py tests/test_gpu_hx.py tests/test_gpu_parity.py} > $O/tests.log 2>&1
s=$?; echo "PYTEST_EXIT $s"; tail -3 $O/tests.log; [ $s -eq 0 ] || exit $s
L=$O/cfg5.txt
for v in 0 16; do
  echo "== GAR_BG_DBG=$v" >> $L
  GAR_BG_DBG=$v P_N=300 timeout -k 10 90 python tools/cfg5_probe.py >> $L 2>&1 || exit 1
done
grep -v amdgpu.ids $L
C=$O/cabi.txt
for w in 4 8; do
  echo "== GAR_HXQ_W=$w" >> $C
  GAR_HXQ_W=$w timeout -k 10 240 ./tools/cabi_stream 4096 30 2 >> $C 2>&1 || exit 1
  GAR_HXQ_W=$w timeout -k 10 240 ./tools/cabi_stream 4096 10 256 >> $C 2>&1 || exit 1
done
cat $C
P=$O/prof.txt
D=$R/go-audio-resampler_amd/libgar_dev.so
for w in 4 8; do
  echo "== GAR_HXQ_W=$w" >> $P
  GAR_HXQ_W=$w GAR_LIB_PATH=$D GAR_HXS_PROF=1 P_N=300 timeout -k 10 90 python tools/stream_probe.py >> $P 2>&1 || exit 1
done
grep -v amdgpu.ids $P | grep -v "loader\|^hxs prof"
