#!/bin/bash
# Round-3 GPU call: GPU tests, smoke, default bench (primary + secondaries + live PMC), one rocprof
# kernel trace of every bench workload, FETCH_SIZE/WRITE_SIZE calibration.  Stops at the first
# failure, fault, abort or timeout.  TAG names the outputs (gpurun_out/<TAG>_*).
TAG=${TAG:-r03a}
O="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$O"
if [ -z "$SKIP_TESTS" ]; then
  # test failures (exit 1) still let the bench run; a crash, abort or timeout ends the call
  timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/${TAG}_gpu_tests.log" 2>&1
  s=$?; echo "PYTEST_EXIT $s" >> "$O/${TAG}_gpu_tests.log"; [ $s -eq 0 ] || [ $s -eq 1 ] || exit $s
  timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > "$O/${TAG}_smoke.log" 2>&1
  s=$?; echo "SMOKE_EXIT $s" >> "$O/${TAG}_smoke.log"; [ $s -eq 0 ] || exit $s
fi
timeout -k 10 900 python -u bench.py $BENCH_ARGS > "$O/${TAG}_bench.log" 2>&1
s=$?; echo "BENCH_EXIT $s" >> "$O/${TAG}_bench.log"; [ $s -eq 0 ] || exit $s
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/${TAG}_prof" -o run -- python "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 3 --no-pmc --no-cpu-baseline --no-streaming --check-seconds 0 > "$O/${TAG}_prof_bench.log" 2>&1
s=$?; echo "PROF_EXIT $s" >> "$O/${TAG}_prof_bench.log"; [ $s -eq 0 ] || exit $s
if [ -z "$SKIP_CALIB" ]; then
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 60 rocprofv3 --pmc $c -d "$O/${TAG}_calib_$c" -o run --output-format csv -- "$GRAFT_REPO_ROOT/tools/ubench/fetch_calib" > "$O/${TAG}_calib_$c.log" 2>&1
    s=$?; echo "CALIB_EXIT $s" >> "$O/${TAG}_calib_$c.log"; [ $s -eq 0 ] || exit $s
  done
fi
exit 0
