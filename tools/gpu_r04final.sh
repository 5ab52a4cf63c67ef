#!/bin/bash
# Round-4 measurement call: all GPU tests, smoke, default bench line, rocprof kernel stats of the
# same command, PMC of the streaming kernels (cfg2 hxs, ns256 hxs, cfg3 hxt), C-ABI short-call numbers.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${FTAG:-r04final}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
s=$?; echo "PYTEST_EXIT $s" >> $O/gpu_tests.log; tail -2 $O/gpu_tests.log; [ $s -eq 0 ] || exit $s
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $O/smoke.log 2>&1
s=$?; echo "SMOKE_EXIT $s" >> $O/smoke.log; tail -1 $O/smoke.log; [ $s -eq 0 ] || exit $s
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
s=$?; echo "BENCH_EXIT $s"; [ $s -eq 0 ] || exit $s
timeout -k 10 240 ./tools/cabi_stream 4096 60 2 > $O/cabi_stereo.txt 2>&1 || exit 1
timeout -k 10 240 ./tools/cabi_stream 4096 10 256 > $O/cabi_256.txt 2>&1 || exit 1
cat $O/cabi_stereo.txt $O/cabi_256.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-pmc > $O/prof_bench.log 2>&1
s=$?; echo "PROF_EXIT $s"; [ $s -eq 0 ] || exit $s
cd $R
TAG=${PT:-r04b}_cfg2 WL=cfg2 KERNEL=hxt_kernel bash tools/pmc_hxs.sh || exit 1
TAG=${PT:-r04b}_ns256 WL=ns256 KERNEL=hxt_kernel bash tools/pmc_hxs.sh || exit 1
TAG=${PT:-r04b}_cfg3 WL=cfg3 KERNEL=hxt_kernel bash tools/pmc_hxs.sh || exit 1
exit 0
