#!/bin/bash
# PMC passes (3) over a python driver script; KERNEL selects the kernel rows summarised.
#   usage: TAG=x KERNEL=poly_kernel bash tools/pmc_generic.sh tools/kone.py
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmcg_${TAG:-x}
mkdir -p $O
S=$R/$1
cd /tmp && export TMPDIR=/tmp
run() { timeout -s KILL 90 rocprofv3 --pmc "$@" -d $O/p$n -o run --output-format csv -- python3 $S > $O/p$n.log 2>&1; }
n=1; run SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU || exit $?
n=2; run SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE || exit $?
python3 $R/tools/pmc_sum.py --kernel ${KERNEL:-poly_kernel} $O > $O/summary.txt 2>&1
cat $O/summary.txt
exit 0
