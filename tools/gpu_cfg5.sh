#!/bin/bash
# cfg5 chunked-path probes: knob variants + one PMC pass over the probe (bg_kernel counters).
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
for v in "" "GAR_BG_DBG=2" "GAR_BG_DBG=1" "GAR_BG_DBG=3"; do
  echo "== $v" >> $O/cfg5_knobs.log
  env $v P_N=300 timeout -k 10 120 python tools/cfg5_probe.py 2>&1 | grep -v "^bg:\|amdgpu.ids\|Exception ignored\|Traceback\|File \|TypeError" >> $O/cfg5_knobs.log || exit $?
done
cd /tmp && export TMPDIR=/tmp
P_N=100 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_MFMA -d $O/pmc_cfg5 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/cfg5_probe.py > $O/pmc_cfg5.log 2>&1 || exit $?
P_N=100 timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM GRBM_GUI_ACTIVE -d $O/pmc_cfg5b -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/cfg5_probe.py > $O/pmc_cfg5b.log 2>&1 || exit $?
exit 0
