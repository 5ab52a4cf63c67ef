#!/bin/bash
# PMC passes over one bench.py workload for the streaming kernels (env knobs pass through).
# WL = workload (cfg2 / ns256 / cfg3), KERNEL = kernel-name filter, TAG names the output dir.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmchxs${TAG}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
S="$R/bench.py --workload ${WL:-cfg2} --steps 3 --warmup 1 --no-cpu-baseline --no-pmc --no-streaming --secondary none --check-seconds 0"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU -d $O/p1 -o run --output-format csv -- python3 $S > $O/p1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d $O/p3 -o run --output-format csv -- python3 $S > $O/p3.log 2>&1 || exit $?
python3 $R/tools/pmc_sum.py --kernel ${KERNEL:-hxs_kernel} $O > $O/summary.txt
cat $O/summary.txt
exit 0
