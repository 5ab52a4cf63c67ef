#!/bin/bash
# Short-call numbers (C-ABI, no Python) with the current defaults + a kernel trace of the stereo stream.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O
TAG=${TAG:-r04d} bash tools/gpu_cabi.sh || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/${TAG:-r04d}_cprof -o run -- $R/tools/cabi_stream 4096 10 2 > $O/${TAG:-r04d}_cprof.log 2>&1 || exit 1
cd $R && python3 tools/prof_db.py $(find $O/${TAG:-r04d}_cprof -name "*.db")
