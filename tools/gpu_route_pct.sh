#!/bin/bash
# Routing share A/B ($PCTVAR: PNP_GYM_WIDE_PCT (default) or PNP_GYM_FULL_PCT, env_dev.h): the gym leg of the bench at each share in
# $PCTS, twice, interleaved.  Each GPU step has its own time limit; the first failure ends it.
set -eu
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
TAG="${TAG:-rp}"
export TMPDIR=/tmp
for i in 1 2; do
  for pc in ${PCTS:-0 50}; do
    env "${PCTVAR:-PNP_GYM_WIDE_PCT}=$pc" timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-tqc --no-ik --no-cpu-baseline > "$OUT/${TAG}_${pc}_$i.log" 2>&1
    echo "pct $pc run $i: $(grep -o '"gym_steps_per_s": [0-9.e+]*' "$OUT/${TAG}_${pc}_$i.log" | head -1) $(grep -o '"max_warn": [0-9]*' "$OUT/${TAG}_${pc}_$i.log" | head -1)"
  done
done
