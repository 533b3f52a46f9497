#!/bin/bash
# Bit-identity check of a refactor: tools/state_digest.py on the current tree and on ab/$TREE
# (default pre), each under its own time limit; prints both digests' differing lines (none = same bits).
set -eu
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
TAG="${TAG:-dg}"
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/state_digest.py ${B:-512} > "$OUT/${TAG}_cur.txt" 2>&1
(cd "$ROOT/ab/${TREE:-pre}" && timeout -k 10 300 python -u tools/state_digest.py ${B:-512}) > "$OUT/${TAG}_ref.txt" 2>&1
grep -v amdgpu "$OUT/${TAG}_cur.txt" | tail -12
if diff <(grep -v amdgpu "$OUT/${TAG}_cur.txt") <(grep -v amdgpu "$OUT/${TAG}_ref.txt") > "$OUT/${TAG}_diff.txt"; then echo "digests identical"; else echo "digests DIFFER"; cat "$OUT/${TAG}_diff.txt"; fi
