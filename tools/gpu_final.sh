#!/bin/bash
# Round-end validation in one GPU call: GPU tests, smoke, bench, rocprof kernel stats of the bench.
# Stops at the first failure, fault, abort or timeout.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
s=$?; echo "PYTEST_EXIT $s" >> gpurun_out/gpu_tests.log; [ $s -eq 0 ] || exit $s
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/smoke.log 2>&1
s=$?; echo "SMOKE_EXIT $s" >> gpurun_out/smoke.log; [ $s -eq 0 ] || exit $s
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1
s=$?; echo "BENCH_EXIT $s" >> gpurun_out/bench.log; [ $s -eq 0 ] || exit $s
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run -- python "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 3 > "$GRAFT_REPO_ROOT/gpurun_out/prof_bench.log" 2>&1
s=$?; echo "PROF_EXIT $s" >> "$GRAFT_REPO_ROOT/gpurun_out/prof_bench.log"; exit $s
