#!/bin/bash
# PMC passes over tools/kone.py (env knobs pass through). TAG names the output dir.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmc1${TAG}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_SMEM SQ_BUSY_CYCLES -d $O/p1 -o run --output-format csv -- python3 $R/tools/kone.py > $O/p1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM GRBM_GUI_ACTIVE -d $O/p2 -o run --output-format csv -- python3 $R/tools/kone.py > $O/p2.log 2>&1 || exit $?
python3 $R/tools/pmc_traffic.py $O x --kernel hx_kernel --write $O/summary.json > /dev/null
exit 0
