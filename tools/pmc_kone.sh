#!/bin/bash
# PMC passes over tools/kone.py for the streaming kernel (KB_* workload env and GAR_* knobs pass
# through).  TAG names the output dir; the summary is gpurun_out/pmck_<TAG>/summary.txt.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmck_${TAG:-x}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
run() { timeout -s KILL 90 rocprofv3 --pmc "$@" -d $O/p$n -o run --output-format csv -- python3 $R/tools/kone.py > $O/p$n.log 2>&1; }
n=1; run SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA || exit $?
n=2; run SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE || exit $?
n=3; run TA_BUSY_avr TA_TA_BUSY_sum SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE || exit $?
python3 $R/tools/pmc_sum.py --kernel ${KERNEL:-hxs_kernel} $O > $O/summary.txt 2>&1
cat $O/summary.txt
exit 0
