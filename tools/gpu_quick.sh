#!/bin/bash
# Quick GPU iteration: gpu tests (all, or $TESTS), stage profile, bench without the CPU leg.
# Each step has its own time limit; the script stops at the first failing step.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
cd "$ROOT"
TAG="${TAG:-quick}"
TESTS="${TESTS:-tests}"
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/${TAG}_pytest.log" 2>&1
rc=$?; tail -3 "$OUT/${TAG}_pytest.log"; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
timeout -k 10 300 python -u tools/step_parity.py 4096 prof > "$OUT/${TAG}_stageprof.log" 2>&1
rc=$?; head -4 "$OUT/${TAG}_stageprof.log"; [ $rc -eq 0 ] || { echo "prof rc=$rc"; exit $rc; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$OUT/${TAG}_bench.log" 2>&1
rc=$?; tail -1 "$OUT/${TAG}_bench.log" | cut -c1-400; exit $rc
