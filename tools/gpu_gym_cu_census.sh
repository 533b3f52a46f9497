#!/bin/bash
# wide-consumer grid (PNP_GYM_QUEUE_CU) sweep: the bench's gym leg per grid in $CUS, then the per-step
# queue census over $NSTEP steps for each grid in $CCUS
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
TAG="${TAG:-cuc}"
export TMPDIR=/tmp
for cu in ${CUS:-4 8 16}; do
  PNP_GYM_QUEUE_CU=$cu timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-tqc --no-ik --no-cpu-baseline > "$OUT/${TAG}_$cu.log" 2>&1 || { tail -5 "$OUT/${TAG}_$cu.log"; exit 1; }
  echo "cu $cu: $(grep -o '"gym_steps_per_s": [0-9.e+]*' "$OUT/${TAG}_$cu.log" | head -1)"
done
for cu in ${CCUS:-8 32}; do
  PNP_GYM_QUEUE_CU=$cu timeout -k 10 300 python -u tools/gym_queue_census.py 4096 ${NSTEP:-10} > "$OUT/${TAG}_census_$cu.log" 2>&1 || { tail -5 "$OUT/${TAG}_census_$cu.log"; exit 1; }
  echo "census cu $cu:"; grep -v amdgpu "$OUT/${TAG}_census_$cu.log" | sed 's/started.*queue {.published.: \([0-9]*\).*next/pub \1 next/' | cut -c1-120
done
