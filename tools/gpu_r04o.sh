#!/bin/bash
# hxt one wave per row block + 6 loaders (GAR_HXT_ROLES=0) vs balanced roles vs hxs, after the spill fixes.
R=${GRAFT_REPO_ROOT:-$(pwd)}
NO_TESTS=1 WORKLOADS="cfg2 ns256" ABS="GAR_HXT=1,GAR_HXT_ROLES=0 GAR_HXT=1 GAR_HXT=0" bash tools/gpu_ab.sh || exit 1
