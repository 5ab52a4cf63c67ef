#!/bin/bash
# Every bench.py workload on one GPU (JSON lines under gpurun_out/), then rocprofv3 kernel stats of each.
R=${GRAFT_REPO_ROOT:-$(pwd)}
D=$R/gpurun_out/${RUN:-r02}; mkdir -p $D
for w in ${WORKLOADS:-cfg2 ns256 cfg3 cfg4 cfg5 pcm16 poly quick}; do
  timeout -k 10 300 python $R/bench.py --workload $w ${BENCH_ARGS:-} > $D/bench_$w.json 2> $D/bench_$w.err || { echo "bench $w failed"; tail -5 $D/bench_$w.err; exit 1; }
  echo "== $w"; tail -c 400 $D/bench_$w.json
done
if [ -z "$NO_PROF" ]; then
  cd /tmp && export TMPDIR=/tmp
  for w in ${WORKLOADS:-cfg2 ns256 cfg3 cfg4 cfg5 pcm16 poly quick}; do
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $D/prof_$w -o run --output-format csv -- python3 $R/bench.py --workload $w --steps 10 --warmup 2 --no-cpu-baseline --no-pmc --no-streaming --check-seconds 0 > $D/prof_$w.log 2>&1 || { echo "prof $w failed"; exit 1; }
  done
fi
exit 0
