#!/bin/bash
# Full -m gpu suite + smoke, then the seeded sweep (tests/test_gpu_sweep.py) for seeds $SEEDS; logs
# under gpurun_out/$TAG.  Stops at the first failure (each step under its own time limit).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-seeds}; mkdir -p $O; cd $R
if [ "${FULL:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
  s=$?; echo "PYTEST_EXIT $s" >> $O/gpu_tests.log; tail -3 $O/gpu_tests.log; [ $s -eq 0 ] || exit $s
  timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
  s=$?; echo "SMOKE_EXIT $s" >> $O/smoke.log; tail -2 $O/smoke.log; [ $s -eq 0 ] || exit $s
fi
for sd in ${SEEDS:-}; do
  GAR_SWEEP_SEED=$sd timeout -k 10 300 python -u -m pytest tests/test_gpu_sweep.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider ${SWEEP_K:+-k "$SWEEP_K"} > $O/seed_$sd.log 2>&1
  s=$?; echo "seed $sd: $(tail -1 $O/seed_$sd.log)" | tee -a $O/seeds.txt; [ $s -eq 0 ] || { tail -40 $O/seed_$sd.log; exit $s; }
done
exit 0
