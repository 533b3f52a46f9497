#!/bin/bash
# C3 step-leg A/B over library variants (VARIANTS: "cur" = pnp_amd/libpnp.so, others
# pnp_amd/libpnp_<v>.so), REPS interleaved rounds; optional gym leg (GYM=1).  Each run has its own
# time limit; stops at the first failure.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
TAG="${TAG:-c3ab}"; LIB=mujoco-panda-pnp_amd/pnp_amd
LEGS="--no-gym --no-tqc --no-ik"; [ -n "${GYM:-}" ] && LEGS="--no-tqc --no-ik"
cp $LIB/libpnp.so /tmp/libpnp_cur.so
for rep in $(seq 1 ${REPS:-2}); do
  for v in ${VARIANTS:-cur base}; do
    if [ $v = cur ]; then cp /tmp/libpnp_cur.so $LIB/libpnp.so; else cp $LIB/libpnp_$v.so $LIB/libpnp.so; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 3 $LEGS --no-cpu-baseline > "$OUT/${TAG}_${v}_$rep.log" 2>&1 || exit $?
    echo "$v $rep: $(grep -o '"value": [0-9.e+]*' "$OUT/${TAG}_${v}_$rep.log" | head -1) $(grep -o '"gym_steps_per_s": [0-9.e+]*' "$OUT/${TAG}_${v}_$rep.log" | head -1)"
  done
done
cp /tmp/libpnp_cur.so $LIB/libpnp.so
