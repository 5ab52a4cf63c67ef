#!/bin/bash
# hxt group size sweep (periods per group) on the default roles.
R=${GRAFT_REPO_ROOT:-$(pwd)}
NO_TESTS=1 WORKLOADS="cfg2 ns256" ABS="GAR_HXS_G=3 GAR_HXS_G=4 -" TRACE=1 bash tools/gpu_ab.sh || exit 1
grep -h "^hxt:" gpurun_out/ab/b_GAR_HXS_G_3_cfg2.err gpurun_out/ab/b_GAR_HXS_G_4_cfg2.err gpurun_out/ab/b_-_cfg2.err | sort | uniq -c | head -8
