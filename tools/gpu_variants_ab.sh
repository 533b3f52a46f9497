#!/bin/bash
# Library variants A/B: tests on pnp_amd/libpnp.so (TESTS), then for each variant (VARIANTS, default
# "cur base": cur = libpnp.so, others pnp_amd/libpnp_<v>.so) the state digest, the bench's C3 step
# and gym legs, and the saturated gym stage profile (slowest envs).  Each GPU step has its own
# time limit; the script stops at the first failure.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
TAG="${TAG:-var}"; LIB=mujoco-panda-pnp_amd/pnp_amd
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 180 --timeout-method thread > "$OUT/${TAG}_pytest.log" 2>&1
  rc=$?; tail -2 "$OUT/${TAG}_pytest.log"; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" "$OUT/${TAG}_pytest.log" | head -20; exit $rc; }
fi
cp $LIB/libpnp.so /tmp/libpnp_cur.so
for v in ${VARIANTS:-cur base}; do
  if [ $v = cur ]; then cp /tmp/libpnp_cur.so $LIB/libpnp.so; else cp $LIB/libpnp_$v.so $LIB/libpnp.so; fi
  timeout -k 10 300 python -u tools/state_digest.py > "$OUT/${TAG}_${v}_digest.log" 2>&1 || exit $?
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-tqc --no-ik --no-cpu-baseline > "$OUT/${TAG}_${v}_bench.log" 2>&1 || exit $?
  echo "$v: $(grep -o '"value": [0-9.e+]*' "$OUT/${TAG}_${v}_bench.log" | head -1) $(grep -o '"gym_steps_per_s": [0-9.e+]*' "$OUT/${TAG}_${v}_bench.log" | head -1) digest $(md5sum < "$OUT/${TAG}_${v}_digest.log" | cut -c1-8)"
  timeout -k 10 300 python -u tools/gym_profile.py 4096 4 saturated > "$OUT/${TAG}_${v}_gymsat.log" 2>&1 || exit $?
  grep -m3 "slow env" "$OUT/${TAG}_${v}_gymsat.log" | cut -c1-200
done
cp /tmp/libpnp_cur.so $LIB/libpnp.so
