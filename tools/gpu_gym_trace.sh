#!/bin/bash
# kernel trace of the bench's gym leg (env as given, e.g. PNP_GYM_HANDBACK=32) + the per-step pass summary
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"
TAG="${TAG:-gtr}"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/${TAG}_prof" -o run -- \
  python3 "$ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-tqc --no-ik > "$OUT/${TAG}.log" 2>&1 || { tail -5 "$OUT/${TAG}.log"; exit 1; }
cd "$ROOT"
f=$(ls "$OUT/${TAG}_prof"/*kernel_trace.csv "$OUT/${TAG}_prof"/*/*kernel_trace.csv 2>/dev/null | head -1)
python3 tools/gym_trace_summary.py "$f" 8 > "$OUT/${TAG}_summary.txt" 2>&1; cat "$OUT/${TAG}_summary.txt"
