#!/bin/bash
# One SQ-counter pass over bench.py (env knobs pass through): TAG names the output dir.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pq${TAG}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
S="$R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --check-seconds 0"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_IFETCH SQ_INSTS_LDS -d $O/p1 -o run --output-format csv -- python3 $S > $O/p1.log 2>&1 || exit $?
python3 - $O/p1/run_counter_collection.csv <<'PY'
import csv, sys, collections
per = collections.defaultdict(float); grid = {}
for r in csv.DictReader(open(sys.argv[1])):
    if 'hxs_kernel' in r['Kernel_Name'] or 'hx_kernel' in r['Kernel_Name']:
        per[(r['Dispatch_Id'], r['Counter_Name'])] += float(r['Counter_Value']); grid[r['Dispatch_Id']] = r.get('Grid_Size', '')
big = max(grid, key=lambda d: per.get((d, 'SQ_WAVE_CYCLES'), 0))
print({c: v for (d, c), v in per.items() if d == big}, 'grid', grid[big])
PY
