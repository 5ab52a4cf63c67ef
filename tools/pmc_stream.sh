#!/bin/bash
# Instruction / scalar cache counters of the streaming (small-launch) hxs kernel.
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P_N=300 timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_HITS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SMEM SQ_WAIT_ANY -d $O/pmc_stream -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/stream_probe.py > $O/pmc_stream.log 2>&1
echo "EXIT $?" >> $O/pmc_stream.log
