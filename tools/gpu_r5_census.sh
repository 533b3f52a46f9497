#!/bin/bash
# round 5: box-box fixture tests, then the BADQACC census: 40 four-step episodes (small / uniform
# actions), and full 300-step episodes with uniform actions (C5's exploration phase) with the
# far-contact check
set -u
OUT=gpurun_out; mkdir -p $OUT/census
TAG=${TAG:-r5c}
timeout -k 10 300 python -u -m pytest tests/test_boxbox_gpu.py -m gpu -v -s --timeout 200 --timeout-method thread > $OUT/${TAG}_box.log 2>&1
rc=$?; tail -4 $OUT/${TAG}_box.log; grep -E "worst error|Error" $OUT/${TAG}_box.log | cut -c1-300; [ $rc -le 1 ] || exit $rc
for pol in small uniform; do
timeout -k 10 400 python -u tools/badqacc_census.py --envs 4096 --episodes 40 --steps 4 --policy $pol --far --out $OUT/census/${pol}_s4.npz > $OUT/${TAG}_census_${pol}_s4.log 2>&1 || { tail -20 $OUT/${TAG}_census_${pol}_s4.log; exit 1; }
tail -20 $OUT/${TAG}_census_${pol}_s4.log
done
timeout -k 10 900 python -u tools/badqacc_census.py --envs 1024 --episodes 4 --steps 300 --policy uniform --probe 5 --far --out $OUT/census/uniform_s300.npz > $OUT/${TAG}_census_uniform_s300.log 2>&1 || { tail -20 $OUT/${TAG}_census_uniform_s300.log; exit 1; }
tail -24 $OUT/${TAG}_census_uniform_s300.log
