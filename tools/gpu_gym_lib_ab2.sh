#!/bin/bash
# library A/B of the bench's gym leg: the in-tree libpnp.so against $ALT (PNP_LIB), interleaved twice
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
TAG="${TAG:-lab}"
export TMPDIR=/tmp
for i in 1 2; do
  for v in tree alt; do
    if [ $v = alt ]; then export PNP_LIB="$ROOT/$ALT"; else unset PNP_LIB; fi
    timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-tqc --no-ik --no-cpu-baseline > "$OUT/${TAG}_${v}_$i.log" 2>&1 || { tail -5 "$OUT/${TAG}_${v}_$i.log"; exit 1; }
    echo "$v run $i: $(grep -o '"gym_steps_per_s": [0-9.e+]*' "$OUT/${TAG}_${v}_$i.log" | head -1)"
  done
done
