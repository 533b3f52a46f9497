#!/bin/bash
# Round-4 GPU iteration: GPU tests ($TESTS, default all), then (only if pytest ended normally:
# pass or test failures, not a fault / abort / timeout) the solver-exit and multiccd diagnostics
# and a bench without the CPU leg.  Each step has its own time limit.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
TAG="${TAG:-r4}"
TESTS="${TESTS:-tests}"
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest $TESTS -m gpu ${PYX--x} -v --timeout 240 --timeout-method thread ${PYK:+-k "$PYK"} > "$OUT/${TAG}_pytest.log" 2>&1
rc=$?; tail -3 "$OUT/${TAG}_pytest.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stop"; exit $rc; fi
prc=$rc
for t in ${DIAGS:-noslip_exit_diag mccd_diag}; do
  timeout -k 10 300 python -u tools/$t.py > "$OUT/${TAG}_$t.log" 2>&1
  rc=$?; echo "== $t rc=$rc"; tail -4 "$OUT/${TAG}_$t.log" | cut -c1-250
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
if [ -z "${NOBENCH:-}" ]; then
  timeout -k 10 400 python -u bench.py --no-cpu-baseline ${BENCHARGS:-} > "$OUT/${TAG}_bench.log" 2>&1
  rc=$?; grep "^\[bench\]" "$OUT/${TAG}_bench.log"; [ $rc -eq 0 ] || exit $rc
fi
exit $prc
