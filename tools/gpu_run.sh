#!/bin/bash
# One measurement call on the GPU box.  Steps (env, 1 = on): TESTS (all -m gpu tests + smoke),
# BENCH (the driver's command: bench.py --gpus 1 --steps 20 --warmup 5), PROF (rocprofv3 kernel
# stats of a short bench run), PMC (PMC passes of the streaming kernel on cfg2 / ns256 / cfg3),
# CABI (C-ABI short-call tool).  TAG names the output dir gpurun_out/$TAG.  Every GPU step runs
# under its own time limit and the script stops at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-run}; mkdir -p $O
cd $R
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 ${TEST_TIMEOUT:-700} python -u -m pytest ${TEST_SEL:-tests} -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
  s=$?; echo "PYTEST_EXIT $s" >> $O/gpu_tests.log; tail -3 $O/gpu_tests.log; [ $s -eq 0 ] || exit $s
  timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $O/smoke.log 2>&1
  s=$?; echo "SMOKE_EXIT $s" >> $O/smoke.log; tail -1 $O/smoke.log; [ $s -eq 0 ] || exit $s
fi
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-500} python3 bench.py --gpus 1 --steps 20 --warmup 5 ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err
  s=$?; echo "BENCH_EXIT $s"; [ $s -eq 0 ] || { tail -20 $O/bench.err; exit $s; }
  python3 - "$O/bench.json" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
def show(k, o):
    r = o.get("roofline", {})
    print(k, round(o["value"]), "kernel_ms", r.get("kernel_ms_per_launch"), r.get("kernel_ms_min_median_max"), "frac", r.get("frac"),
          "traffic/algo", r.get("traffic_over_algo"), "rms", o.get("rms_vs_oracle"))
show("cfg2", d)
for k, o in (d.get("secondary") or {}).items():
    show(k, o)
print("stream", d.get("stream_dev_us_per_call"), d.get("stream_host_us_per_call"), d.get("stream_256ch_host_ms_per_call"),
      "cpu", d.get("cpu_baseline_msamples_per_s"), d.get("cpu_baseline_cores"))
EOF
fi
if [ "${CABI:-0}" = 1 ]; then
  timeout -k 10 240 ./tools/cabi_stream 4096 60 2 > $O/cabi_stereo.txt 2>&1 || exit 1
  timeout -k 10 240 ./tools/cabi_stream 4096 10 256 > $O/cabi_256.txt 2>&1 || exit 1
  tail -n 3 $O/cabi_stereo.txt $O/cabi_256.txt
fi
if [ "${PROF:-1}" = 1 ]; then
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-pmc > $O/prof_bench.log 2>&1 )
  s=$?; echo "PROF_EXIT $s"; [ $s -eq 0 ] || exit $s
  f=$(find $O/prof -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && head -12 "$f"
fi
if [ "${PMC:-1}" = 1 ]; then
  for w in ${PMC_WL:-cfg2 ns256 cfg3}; do
    TAG=${TAG:-run}_$w WL=$w KERNEL=${PMC_KERNEL:-hxt_kernel} bash tools/pmc_hxs.sh > /dev/null || exit 1
    echo "== PMC $w"; cat $R/gpurun_out/pmchxs${TAG:-run}_$w/summary.txt
  done
fi
exit 0
