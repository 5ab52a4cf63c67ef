O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P_N=100 timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_REQ SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY -d $O/pmc_ic -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/cfg5_probe.py > $O/pmc_ic.log 2>&1
echo "EXIT $?" >> $O/pmc_ic.log
