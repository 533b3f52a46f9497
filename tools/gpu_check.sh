#!/bin/bash
# GPU pass after a kernel change: gpu tests (all or $TESTS), bench (no CPU leg), gym profile.
# Each step has its own time limit; the script stops at the first failing step.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
cd "$ROOT"
TAG="${TAG:-chk}"
TESTS="${TESTS:-tests}"
timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v --timeout 180 --timeout-method thread > "$OUT/${TAG}_pytest.log" 2>&1
rc=$?; tail -3 "$OUT/${TAG}_pytest.log"; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; grep -E "FAILED|Error" "$OUT/${TAG}_pytest.log" | head; exit $rc; }
timeout -k 10 400 python -u bench.py --no-cpu-baseline > "$OUT/${TAG}_bench.log" 2>&1
rc=$?; tail -1 "$OUT/${TAG}_bench.log" | cut -c1-300; [ $rc -eq 0 ] || exit $rc
if [ -n "${GYM:-}" ]; then
  timeout -k 10 300 python -u tools/gym_profile.py 4096 4 uniform > "$OUT/${TAG}_gym_uniform.log" 2>&1 || exit $?
  timeout -k 10 300 python -u tools/gym_profile.py 4096 4 saturated > "$OUT/${TAG}_gym_sat.log" 2>&1 || exit $?
fi
echo "done"
