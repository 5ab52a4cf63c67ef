#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
export GAR_LIB_PATH=$R/go-audio-resampler_amd/libgar_dev.so
TAG=r06t MODES="0 16 4 20 1" WL=ns256 bash tools/gpu_dbg_modes.sh || exit 1
for m in 0 16 4; do
  GAR_HXS_DBG=$m TAG=r06t_m$m WL=ns256 KERNEL=hxt_kernel bash tools/pmc_hxs.sh > /dev/null || exit 1
  echo "== mode $m"; cat gpurun_out/pmchxsr06t_m$m/summary.txt
done
