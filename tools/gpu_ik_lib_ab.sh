#!/bin/bash
# IK A/B of two library builds: IK + skill GPU tests on the tree's libpnp.so, then the C2 bench
# leg (both regimes) on it and on pnp_amd/libpnp_$VARIANT.so swapped in.  Each GPU step has its
# own time limit; the script stops at the first failing step.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
LIB=mujoco-panda-pnp_amd/pnp_amd; V="${VARIANT:-ik8}"
timeout -k 10 300 python -u -m pytest tests/test_ik_gpu.py tests/test_skills_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/ikab_pytest.log" 2>&1
rc=$?; tail -3 "$OUT/ikab_pytest.log"; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" "$OUT/ikab_pytest.log" | head -20; exit $rc; }
cp $LIB/libpnp.so /tmp/libpnp_new.so
for v in new $V new $V; do
  cp /tmp/libpnp_$v.so $LIB/libpnp.so 2>/dev/null || cp $LIB/libpnp_$v.so $LIB/libpnp.so
  for r in waypoint ik_test; do
    extra=""; [ $r = ik_test ] && extra="--params ik_test"
    timeout -k 10 200 python -u bench.py --workload ik --regime $r $extra --steps 500 --warmup 20 --no-cpu-baseline > "$OUT/ikab_${v}_$r.log" 2>&1 || exit $?
    tail -1 "$OUT/ikab_${v}_$r.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v $r', round(d['value']/1e6,2), 'M solves/s', round(d['ms_per_step']*1e3,1), 'us', d['ik_stats'])"
  done
done
cp /tmp/libpnp_new.so $LIB/libpnp.so
