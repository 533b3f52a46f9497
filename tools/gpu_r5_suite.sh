#!/bin/bash
# round 5: the whole GPU suite (per-tree bars printed), then the stage profile and a bench without CPU leg
set -u
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-r5s}
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $OUT/${TAG}_pytest.log 2>&1
rc=$?; tail -5 $OUT/${TAG}_pytest.log; grep -E "FAILED|worst error" $OUT/${TAG}_pytest.log | cut -c1-300 | head -30; [ $rc -le 1 ] || exit $rc
if [ -n "${PROF:-}" ]; then
timeout -k 10 300 python -u tools/step_parity.py 4096 prof bench > $OUT/${TAG}_stageprof.log 2>&1 || exit $?
head -40 $OUT/${TAG}_stageprof.log | grep -E "M env|per env|newton|n_" 
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $OUT/${TAG}_bench.log 2>&1 || exit $?
tail -1 $OUT/${TAG}_bench.log | cut -c1-300
fi
