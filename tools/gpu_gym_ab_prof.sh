#!/bin/bash
# Gym-state stage profile, current tree against ab/$TREE (default v19): tools/gym_profile.py on
# 4096 envs after 4 random-action gym steps, each tree in turn.  Each GPU step has its own limit.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
TAG="${TAG:-gab}"
export TMPDIR=/tmp
for t in cur ${TREE:-v19}; do
  d="$ROOT"; [ "$t" = cur ] || d="$ROOT/ab/$t"
  (cd "$d" && timeout -k 10 240 python -u tools/gym_profile.py 4096 4 ${MODE:-uniform}) > "$OUT/${TAG}_${t}.log" 2>&1 || exit $?
  echo "$t: $(grep -m1 "cycles" "$OUT/${TAG}_${t}.log")"
done
