#!/bin/bash
# Kernel timing protocol A/B: library HIP events inside the timed region (default) vs a separate
# profiled pass, each beside a rocprofv3 kernel trace of the same command.
R=${GRAFT_REPO_ROOT:-$(pwd)}; D=$R/gpurun_out/profab; mkdir -p $D
cd /tmp && export TMPDIR=/tmp
for inl in 1 0; do
  GAR_BENCH_PROF_INLINE=$inl timeout -k 10 120 python3 $R/bench.py --no-cpu-baseline --no-pmc --no-streaming > $D/bench_$inl.json 2>/dev/null || exit 1
  GAR_BENCH_PROF_INLINE=$inl timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $D/prof_$inl -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-pmc --no-streaming --check-seconds 0 > $D/prof_$inl.log 2>&1 || exit 1
done
for inl in 1 0; do
  python3 -c "import json; d=json.loads(open('$D/bench_$inl.json').read().strip().splitlines()[-1]); print('inline=$inl', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_launch'])"
  python3 $R/tools/trace_summary.py $(find $D/prof_$inl -name '*kernel_trace.csv' | head -1) | head -2
done
