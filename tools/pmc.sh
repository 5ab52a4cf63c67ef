#!/bin/bash
# Kernel trace + PMC passes of bench.py (separate passes; never combined with other trace domains).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/prof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --steps ${PROF_STEPS:-20} --warmup 2 --no-cpu-baseline --check-seconds 0"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- $B > $O/trace.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES -d $O/p1 -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --check-seconds 0 > $O/p1.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc GRBM_GUI_ACTIVE FETCH_SIZE -d $O/p2 -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --check-seconds 0 > $O/p2.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $O/p3 -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --check-seconds 0 > $O/p3.log 2>&1 || exit $?
python3 $R/tools/pmc_traffic.py $O cfg2_stereo_f32_44k1_48k_q24_600s --write $O/pmc_summary.json > /dev/null
exit 0
