#!/bin/bash
# env-variable A/B of the bench's C5 (TQC) leg: $VAR at each value in $VALS, interleaved twice
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
TAG="${TAG:-tlab}"
export TMPDIR=/tmp
for i in 1 2; do
  for v in $VALS; do
    env "$VAR=$v" timeout -k 10 400 python -u bench.py --steps 5 --warmup 1 --no-gym --no-ik --no-cpu-baseline > "$OUT/${TAG}_${v}_$i.log" 2>&1 || { tail -5 "$OUT/${TAG}_${v}_$i.log"; exit 1; }
    python3 - "$OUT/${TAG}_${v}_$i.log" "$VAR=$v run $i" <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
t = json.loads(l)["tqc"]
print(sys.argv[2], "tqc %.0f transitions/s, %.1f ms per step, UTD %.0f (%.1f ms per vector step)" % (
    t["gym_steps_per_s"], t["ms_per_step"], t["transitions_per_s_at_reference_utd"], t["reference_utd"]["ms_per_vector_step"]))
PY
  done
done
