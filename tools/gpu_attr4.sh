#!/bin/bash
# hxt attribution on the dev build: DBG modes (1 no steady loads, 2 no stores, 4 no MFMA, 16 no conversion).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/attr; mkdir -p $O
D=$R/go-audio-resampler_amd/libgar_dev.so
for wl in "KB_CH=2 KB_SECONDS=600" "KB_CH=256 KB_SECONDS=60"; do
  tag=$(echo $wl | cut -d' ' -f1 | tr '=' '_')
  env $wl timeout -k 10 300 python tools/kbench.py "[{\"GAR_LIB_PATH\":\"$D\"},{\"GAR_LIB_PATH\":\"$D\",\"GAR_HXS_DBG\":\"4\"},{\"GAR_LIB_PATH\":\"$D\",\"GAR_HXS_DBG\":\"2\"},{\"GAR_LIB_PATH\":\"$D\",\"GAR_HXS_DBG\":\"16\"},{\"GAR_LIB_PATH\":\"$D\",\"GAR_HXS_DBG\":\"17\"},{\"GAR_LIB_PATH\":\"$D\",\"GAR_HXS_DBG\":\"6\"},{\"GAR_LIB_PATH\":\"$D\",\"GAR_HXS_DBG\":\"19\"},{\"GAR_LIB_PATH\":\"$D\",\"GAR_HXS_DBG\":\"23\"},{\"GAR_LIB_PATH\":\"$D\",\"GAR_HXT\":\"0\"},{\"GAR_LIB_PATH\":\"$D\",\"GAR_HXT\":\"0\",\"GAR_HXS_DBG\":\"4\"}]" > $O/$tag.jsonl 2>&1 || exit 1
  cat $O/$tag.jsonl
done
