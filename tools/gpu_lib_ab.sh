#!/bin/bash
# Library A/B on the step workload: the C3 step leg and the stage-cycle profile with
# pnp_amd/libpnp.so, then with each pnp_amd/libpnp_<variant>.so swapped in (VARIANTS="inl ...");
# a variant's GPU tests (TESTS, default the step parity tests) run before it is timed.  Each GPU step has its own time limit.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
TAG="${TAG:-lab}"; LIB=mujoco-panda-pnp_amd/pnp_amd
cp $LIB/libpnp.so /tmp/libpnp_base.so
for v in base ${VARIANTS:-inl}; do
  if [ $v != base ]; then
    cp $LIB/libpnp_$v.so $LIB/libpnp.so
    timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_step_gpu.py} -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/${TAG}_${v}_pytest.log" 2>&1
    rc=$?; tail -2 "$OUT/${TAG}_${v}_pytest.log"; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" "$OUT/${TAG}_${v}_pytest.log" | head -20; exit $rc; }
  fi
  for i in 1 2; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 3 ${BENCH_ARGS:---no-gym --no-tqc --no-ik} --no-cpu-baseline > "$OUT/${TAG}_${v}_bench$i.log" 2>&1 || exit $?
    echo "$v run $i: $(grep -o '"value": [0-9.e+]*' "$OUT/${TAG}_${v}_bench$i.log" | head -1) $(grep -o '"gym_steps_per_s": [0-9.e+]*' "$OUT/${TAG}_${v}_bench$i.log" | head -1)"
  done
  timeout -k 10 300 python3 -u tools/step_parity.py 4096 prof > "$OUT/${TAG}_${v}_stageprof.log" 2>&1 || exit $?
  grep -m1 "cycles" "$OUT/${TAG}_${v}_stageprof.log"
done
cp /tmp/libpnp_base.so $LIB/libpnp.so
