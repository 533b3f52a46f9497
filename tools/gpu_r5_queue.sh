#!/bin/bash
# round 5: hand-over queue fallback / two-stream tests, per-tree fp32 bars, gloo 2-rank bench record
set -u
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-r5q}
timeout -k 10 500 python -u -m pytest tests/test_env_gpu.py -m gpu -v -s --timeout 200 --timeout-method thread -k "queue or in_flight or routing or compact_tier" > $OUT/${TAG}_env.log 2>&1
rc=$?; tail -3 $OUT/${TAG}_env.log; grep "queue status" $OUT/${TAG}_env.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_step_gpu.py -m gpu -v -s --timeout 300 --timeout-method thread -k "per_tree or wide_tier or mesh or multiccd" > $OUT/${TAG}_step.log 2>&1
rc=$?; tail -3 $OUT/${TAG}_step.log; grep -E "floor per tree|worst error" $OUT/${TAG}_step.log | cut -c1-400; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 --no-gym --no-tqc --no-ik --no-cpu-baseline > $OUT/${TAG}_gloo2.log 2>&1 || { tail -30 $OUT/${TAG}_gloo2.log; exit 1; }
tail -1 $OUT/${TAG}_gloo2.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['value'], json.dumps(r['dist']))"
mkdir -p $OUT/census
timeout -k 10 400 python -u tools/badqacc_census.py --envs 4096 --episodes 40 --steps 4 --policy small --out $OUT/census/small_s4.npz > $OUT/${TAG}_census_small.log 2>&1 || { tail -20 $OUT/${TAG}_census_small.log; exit 1; }
tail -22 $OUT/${TAG}_census_small.log
timeout -k 10 400 python -u tools/badqacc_census.py --envs 4096 --episodes 40 --steps 4 --policy uniform --out $OUT/census/uniform_s4.npz > $OUT/${TAG}_census_uniform.log 2>&1 || { tail -20 $OUT/${TAG}_census_uniform.log; exit 1; }
tail -22 $OUT/${TAG}_census_uniform.log
