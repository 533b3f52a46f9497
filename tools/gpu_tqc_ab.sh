#!/bin/bash
# fused learner A/B on the GPU box: the fused tests, learner-step timing, a kernel trace of the
# learner step.  Each GPU step under its own limit; stops at the first failure.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
TAG="${TAG:-tqcab}"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_tqc_gpu.py -k fused > "$OUT/${TAG}_tests.log" 2>&1 || { tail -20 "$OUT/${TAG}_tests.log"; exit 1; }
tail -1 "$OUT/${TAG}_tests.log"
timeout -k 10 120 python3 tools/tqc_learner_bench.py fused 300 > "$OUT/${TAG}_bench.log" 2>&1 || { tail -5 "$OUT/${TAG}_bench.log"; exit 1; }
grep fused "$OUT/${TAG}_bench.log" | cut -c1-90
cd /tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_trace" -o run -- python3 "$ROOT/tools/tqc_learner_bench.py" fused 200 > "$OUT/${TAG}_trace.log" 2>&1 || { tail -5 "$OUT/${TAG}_trace.log"; exit 1; }
f=$(ls "$OUT/${TAG}_trace"/*/*kernel_stats.csv 2>/dev/null | head -1)
[ -n "$f" ] || f=$(ls "$OUT/${TAG}_trace"/*kernel_stats.csv | head -1)
cut -d, -f1-5 "$f" | grep -i tqc | cut -c1-140
