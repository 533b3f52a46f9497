#!/bin/bash
# Library A/B on the gym workload: for pnp_amd/libpnp.so ("new") and pnp_amd/libpnp_base.so
# ("base"), interleaved twice: the bench's gym leg (4096 envs, random actions) and the heavy-env
# stage profile (tools/gym_profile.py, saturated actions).  Tests (TESTS) run on the new library
# first.  Each GPU step has its own time limit; stops at the first failure.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
TAG="${TAG:-glab}"; LIB=mujoco-panda-pnp_amd/pnp_amd
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 180 --timeout-method thread > "$OUT/${TAG}_pytest.log" 2>&1
  rc=$?; tail -2 "$OUT/${TAG}_pytest.log"; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" "$OUT/${TAG}_pytest.log" | head -20; exit $rc; }
fi
cp $LIB/libpnp.so /tmp/libpnp_new.so
for rep in 1 2; do
  for v in new base; do
    if [ $v = base ]; then cp $LIB/libpnp_base.so $LIB/libpnp.so; else cp /tmp/libpnp_new.so $LIB/libpnp.so; fi
    timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-tqc --no-ik --no-cpu-baseline > "$OUT/${TAG}_${v}_bench$rep.log" 2>&1 || exit $?
    echo "$v run $rep: $(grep -o '"gym_steps_per_s": [0-9.e+]*' "$OUT/${TAG}_${v}_bench$rep.log" | head -1) $(grep -o '"value": [0-9.e+]*' "$OUT/${TAG}_${v}_bench$rep.log" | head -1)"
    if [ $rep = 1 ]; then
      timeout -k 10 300 python -u tools/gym_profile.py 4096 4 saturated > "$OUT/${TAG}_${v}_gymsat.log" 2>&1 || exit $?
    fi
  done
done
cp /tmp/libpnp_new.so $LIB/libpnp.so
