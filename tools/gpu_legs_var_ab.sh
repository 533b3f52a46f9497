#!/bin/bash
# env-variable A/B of the bench's gym and C5 legs: $VAR at each value in $VALS, interleaved twice
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
TAG="${TAG:-lvab}"
export TMPDIR=/tmp
for i in 1 2; do
  for v in $VALS; do
    env "$VAR=$v" timeout -k 10 400 python -u bench.py --steps 5 --warmup 1 --no-ik --no-cpu-baseline > "$OUT/${TAG}_${v}_$i.log" 2>&1 || { tail -5 "$OUT/${TAG}_${v}_$i.log"; exit 1; }
    python3 - "$OUT/${TAG}_${v}_$i.log" "$VAR=$v run $i" <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[1]) if x.startswith("{")][-1])
g, t = d["gym"], d["tqc"]
print(sys.argv[2], "gym %.0f (%.1f ms)  C5 %.0f transitions/s, UTD %.0f" % (
    g["gym_steps_per_s"], g["ms_per_gym_step"], t["gym_steps_per_s"], t["transitions_per_s_at_reference_utd"]))
PY
  done
done
