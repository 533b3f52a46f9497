#!/bin/bash
# Gym-step routing check: env / TQC / step GPU tests, the bench gym leg with routing off and on,
# and a kernel trace of the routed gym leg (tools/gym_trace_summary.py).  Each GPU step has its
# own time limit; the script stops at the first failure.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
TAG="${TAG:-route}"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_env_gpu.py tests/test_tqc_gpu.py tests/test_step_gpu.py -m gpu -x -q --timeout 180 --timeout-method thread > "$OUT/${TAG}_pytest.log" 2>&1
rc=$?; tail -3 "$OUT/${TAG}_pytest.log"; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" "$OUT/${TAG}_pytest.log" | head -20; exit $rc; }
for r in 0 1; do
  PNP_GYM_ROUTE=$r timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-tqc --no-ik --no-cpu-baseline > "$OUT/${TAG}_bench_r$r.log" 2>&1 || exit $?
  echo "route=$r: $(grep -o '"gym_steps_per_s": [0-9.e+]*' "$OUT/${TAG}_bench_r$r.log")  C3 $(grep -o '"value": [0-9.e+]*' "$OUT/${TAG}_bench_r$r.log" | head -1)"
done
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_trace" -o run -- python3 "$ROOT/bench.py" --steps 10 --warmup 2 --no-tqc --no-ik --no-cpu-baseline > "$OUT/${TAG}_trace.log" 2>&1 || exit $?
cd "$ROOT"
python3 tools/gym_trace_summary.py "$(find "$OUT/${TAG}_trace" -name '*kernel_trace.csv' | head -1)" 12
