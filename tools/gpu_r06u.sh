#!/bin/bash
# r06u: split bit check, mixed-precision split A/B (3 rounds), compile-time attribution of hxt_kernel
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out/r06u
timeout -k 10 120 ./tools/ubench/split_check 1 > gpurun_out/r06u/split_check.txt 2>&1 || { cat gpurun_out/r06u/split_check.txt; exit 1; }
cat gpurun_out/r06u/split_check.txt
TAG=r06u_ab LIBS="libgar.so libgar_mix.so" WL=ns256 SEC=cfg2,cfg3 ROUNDS=3 bash tools/ab_bench.sh || exit 1
TAG=r06u_attr LIBS="libgar.so libgar_ct2.so libgar_ct16.so libgar_ct4.so libgar_ct12.so libgar_ct20.so" WL=ns256 SEC=cfg2 ROUNDS=1 bash tools/ab_bench.sh || exit 1
