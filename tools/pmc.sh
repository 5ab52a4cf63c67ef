#!/bin/bash
# Kernel trace + PMC passes of bench.py (separate passes; never combined with other trace domains).
# KERNEL (default hx_kernel) = the dominant kernel summarised; PROF_TAG names the output dir.
R=${GRAFT_REPO_ROOT:-$(pwd)}
K=${KERNEL:-hx_kernel}
O=$R/gpurun_out/prof${PROF_TAG}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps ${PROF_STEPS:-20} --warmup 2 --no-cpu-baseline --check-seconds 0"
S="$R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --check-seconds 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $B > $O/trace.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_VALU -d $O/p1 -o run --output-format csv -- python3 $S > $O/p1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE FETCH_SIZE -d $O/p2 -o run --output-format csv -- python3 $S > $O/p2.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_MFMA -d $O/p3 -o run --output-format csv -- python3 $S > $O/p3.log 2>&1 || exit $?
python3 $R/tools/pmc_traffic.py $O cfg2_stereo_f32_44k1_48k_q24_600s --kernel $K --write $O/pmc_summary.json > /dev/null
python3 $R/tools/trace_summary.py $O/trace/run_kernel_trace.csv --write $O/trace_by_grid.json > $O/trace_by_grid.txt
exit 0
